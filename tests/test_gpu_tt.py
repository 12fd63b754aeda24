"""GPU: the temperature-only pixel path (gibbssampler_amd.tt, row f4) through
the reference's class surface, replay mode against the reference's own TT
numbers (tools/gen_golden_tt.py) and native mode against the oracle chains."""
import os

import numpy as np
import pytest

from oracle import harmonic as H
from oracle import masked as MK

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_tt_N8_L16.npz")


@pytest.fixture(scope="module")
def g():
    return dict(np.load(GOLDEN))


def _close(a, b, rtol=1e-9):
    np.testing.assert_allclose(a, b, rtol=rtol, atol=1e-11 * np.abs(b).max())


def _args(g):
    N, L = int(g["nside"]), int(g["L"])
    noise = np.full(12 * N * N, float(g["noise"]))
    return N, L, noise


def _centered(g, **kw):
    from gibbssampler_amd.gibbs import CenteredGibbs
    N, L, noise = _args(g)
    return CenteredGibbs(g["T"], noise, noise, float(g["fwhm_deg"]), N, L, 12 * N * N, polarization=False,
                         bins=g["bins"], **kw)


def _nc(g, **kw):
    from gibbssampler_amd.gibbs import NonCenteredGibbs
    N, L, noise = _args(g)
    return NonCenteredGibbs(g["T"], noise, noise, float(g["fwhm_deg"]), N, L, 12 * N * N, g["pv"],
                            metropolis_blocks=g["blocks"], polarization=False, bins=g["bins"], **kw)


def _asis(g, **kw):
    from gibbssampler_amd.gibbs import ASIS
    N, L, noise = _args(g)
    return ASIS(g["T"], noise, noise, float(g["fwhm_deg"]), N, L, 12 * N * N, g["pv"], metropolis_blocks=g["blocks"],
                polarization=False, bins=g["bins"], **kw)


def _var(g):
    from gibbssampler_amd import utils
    return utils.generate_var_cl(g["dl_TT"])


def test_fullsky_cr_replay(g):
    cg = _centered(g, n_iter=1, rng="replay")
    assert cg.tt_pixel
    np.random.seed(int(g["cr_c_seed"]))
    s, acc = cg.constrained_sampler.sample(None, _var(g), None)
    assert acc == 1
    _close(s, g["cr_c"])
    nc = _nc(g, n_iter=1, rng="replay")
    np.random.seed(int(g["cr_nc_seed"]))
    s, _ = nc.constrained_sampler.sample(None, _var(g), None, False)
    _close(s, g["cr_nc"])


def test_aux_replay(g):
    cg = _centered(g, n_iter=1, rng="replay", mask_path=g["mask"])
    np.random.seed(int(g["aux_seed"]))
    s, acc = cg.constrained_sampler.sample(None, _var(g), g["aux_s_old"], use_gibbs=True)
    assert acc == 1
    _close(s, g["aux_out"])


def test_cls_replay(g):
    cg = _centered(g, n_iter=1, rng="replay")
    np.random.seed(int(g["cls_seed"]))
    _close(cg.cls_sampler.sample(g["cr_c"]), g["cls_out"])


@pytest.mark.parametrize("tag", ["mh", "mhm"])
def test_pixel_mh_replay(g, tag):
    from gibbssampler_amd import utils
    nc = _nc(g, n_iter=1, rng="replay", mask_path=(g["mask"] if tag == "mhm" else None))
    var0 = utils.generate_var_cl(utils.unfold_bins(g["init"], g["bins"]))
    assert nc.cls_sampler.compute_log_likelihood(var0, g["mh_snc"]) == pytest.approx(float(g[tag + "_lik0"]),
                                                                                      rel=1e-11)
    np.random.seed(int(g[tag + "_seed"]))
    b, var, acc = nc.cls_sampler.sample(g["mh_snc"], g["init"].copy(), var0)
    _close(b, g[tag + "_out"])
    assert list(acc) == list(g[tag + "_accept"])
    assert var.shape == var0.shape


@pytest.mark.parametrize("key", ["drv_c", "drv_nc", "drv_asis", "drv_asisg"])
def test_drivers_replay(g, key):
    n = int(g["drv_iters"])
    if key == "drv_c":
        smp = _centered(g, n_iter=n, rng="replay")
    elif key == "drv_nc":
        smp = _nc(g, n_iter=n, rng="replay")
    else:
        smp = _asis(g, n_iter=n, rng="replay", gibbs_cr=(key == "drv_asisg"))
    np.random.seed(int(g[key + "_seed"]))
    out = smp.run(g["init"].copy())
    _close(out[0], g[key + "_h"])
    if key != "drv_c":
        np.testing.assert_array_equal(out[1], g[key + "_acc"])
    if key.startswith("drv_asis"):
        assert len(out) == 4 and np.all(out[2] == 1)


def _oracle_native(g, kind, seed, masked=False, gcr=False):
    L = int(g["L"])
    Npix = int(g["Npix"])
    inv = np.full(Npix, 1.0 / float(g["noise"])) * (g["mask"] if masked else 1.0)
    mm = MK.tt_model(L, int(g["nside"]), g["bl"], g["T"], inv)
    model = H.Model(L, int(g["nside"]), 1, g["bl"], [1.0], {"TT": g["bins"]}, blocks={"TT": g["blocks"]},
                    proposal_variances={"TT": g["pv"]}, d_alm=np.zeros((1, (L + 1) ** 2)))
    return MK.tt_chain(kind, mm, mm, model, {"TT": g["init"]}, 3,
                       lambda it: MK.NativeDraws(seed, 0, it, L, Npix), gibbs_cr=gcr, native=(seed, 0))


@pytest.mark.parametrize("kind,masked,gcr", [("centered", False, False), ("noncentered", False, False),
                                             ("asis", False, True), ("centered", True, False),
                                             ("noncentered", True, False)])
def test_drivers_native_vs_oracle(g, kind, masked, gcr):
    seed = 31
    mp = g["mask"] if masked else None
    if kind == "centered":
        smp = _centered(g, n_iter=3, rng="native", seed=seed, mask_path=mp)
    elif kind == "noncentered":
        smp = _nc(g, n_iter=3, rng="native", seed=seed, mask_path=mp)
    else:
        smp = _asis(g, n_iter=3, rng="native", seed=seed, gibbs_cr=gcr, mask_path=mp)
    if masked:
        smp._tt.cr.pcg_accuracy = 1e-13
    out = smp.run(g["init"].copy())
    want, wacc, _ = _oracle_native(g, kind, seed, masked, gcr)
    _close(out[0], want, rtol=1e-8)
    if kind != "centered":
        np.testing.assert_array_equal(out[1], wacc)
