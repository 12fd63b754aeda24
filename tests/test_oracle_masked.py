"""CPU: the masked-CR oracle (oracle/masked.py) against golden vectors produced
by the reference itself (tools/gen_golden_masked.py, SHT served by oracle/sht).

Pins the auxiliary-variable (a9), over-relaxation (a10) and MALA (a11)
samplers, the dispatch composition (a12) and a 3-iteration masked centered
driver, in the reference's numpy draw order."""
import os

import numpy as np
import pytest

from oracle import harmonic as H
from oracle import masked as MK
from oracle import reference_eb as RE

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_masked_eb_N8_L16.npz")


@pytest.fixture(scope="module")
def g():
    return dict(np.load(GOLDEN))


def _mm(g):
    L, N = int(g["L"]), int(g["nside"])
    Npix = 12 * N * N
    maps = np.stack([np.zeros(Npix), g["Q"], g["U"]])
    inv = np.stack([np.zeros(Npix), g["inv_noise_pol"], g["inv_noise_pol"]])
    return MK.MaskedModel(L, N, 2, g["bl"], maps, inv)


def _dl(g):
    return np.stack([g["dl_EE"], g["dl_BB"]])


def _s_old(g):
    return np.stack([g["s_old_E"], g["s_old_B"]])


def _close(a, b):
    np.testing.assert_allclose(a, b, rtol=1e-10, atol=1e-12 * np.abs(b).max())


def test_constants(g):
    mm = _mm(g)
    th, _ = __import__("oracle.sht", fromlist=["x"]).pixel_angles(int(g["nside"]))
    np.testing.assert_array_equal(g["mask"], (np.abs(np.cos(th)) > 0.2).astype(float))
    np.testing.assert_allclose(g["inv_noise_pol"], g["mask"] / g["noise_pol"], rtol=1e-15)
    assert mm.mu[1] == pytest.approx(float(g["mu"]), rel=1e-15)
    g2 = mm.second_part_grad()
    _close(g2[0], g["second_part_grad_E"])
    _close(g2[1], g["second_part_grad_B"])


def test_a9_aux_variable(g):
    s, acc = MK.aux_variable(_mm(g), _dl(g), _s_old(g), int(g["a9_ngibbs"]), MK.ReplayDraws(int(g["a9_seed"])))
    assert acc == int(g["a9_accept"]) == 1
    _close(s[0], g["a9_E"])
    _close(s[1], g["a9_B"])


def test_a10_overrelaxation(g):
    s, acc = MK.overrelaxation(_mm(g), _dl(g), _s_old(g), int(g["a10_ngibbs"]), MK.ReplayDraws(int(g["a10_seed"])),
                               alpha=float(g["a10_alpha"]))
    assert acc == 1
    _close(s[0], g["a10_E"])
    _close(s[1], g["a10_B"])


def test_a11_gradient(g):
    mm = _mm(g)
    grad, pix = MK.mala_gradient(mm, _dl(g), _s_old(g), mm.second_part_grad())
    _close(grad[0], g["a11_gradE"])
    _close(grad[1], g["a11_gradB"])
    _close(pix[0], g["a11_sEpix"])
    _close(pix[1], g["a11_sBpix"])


@pytest.mark.parametrize("variant", ["a11", "a11b"])
def test_a11_mala(g, variant):
    mm = _mm(g)
    start = _s_old(g) if variant == "a11" else np.stack([g["a9_E"], g["a9_B"]])
    tau = float(g["a11_tau"]) if variant == "a11" else float(g["a11b_tau"])
    for k, sd in enumerate(g[variant + "_seeds"]):
        s, acc, _ = MK.mala(mm, _dl(g), start, MK.ReplayDraws(int(sd)), float(g["noise_pol"][0]), tau=tau)
        assert acc == int(g[variant + "_accept"][k])
        _close(s[0], g[variant + "_E"][k])
        _close(s[1], g[variant + "_B"][k])


def test_a12_composition(g):
    s, acc = MK.sample_dispatch(_mm(g), _dl(g), _s_old(g), MK.ReplayDraws(int(g["a12_seed"])), gibbs_cr=True,
                                overrelaxation_flag=False, ula=True, n_gibbs=int(g["a12_ngibbs"]),
                                noise_pol0=float(g["noise_pol"][0]))
    assert acc == int(g["a12_accept"])
    _close(s[0], g["a12_E"])
    _close(s[1], g["a12_B"])


def test_masked_centered_driver(g):
    """CenteredGibbs.run_polarization (GibbsSampler.py:118-180) with the a9 CR and
    the injected start map; C_l draws in the reference's invgamma order."""
    mm = _mm(g)
    L = int(g["L"])
    bins = {"EE": g["bins_EE"], "BB": g["bins_BB"]}
    model = H.Model(L, int(g["nside"]), 2, g["bl"], [1.0, 1.0], bins, d_alm=np.zeros((2, (L + 1) ** 2)))
    np.random.seed(int(g["drv_seed"]))
    binned = {"EE": g["init_EE"].copy(), "BB": g["init_BB"].copy()}
    hist = {"EE": [binned["EE"]], "BB": [binned["BB"]]}
    skymap = _s_old(g)
    draws = MK.ReplayDraws()
    for _ in range(int(g["drv_iters"])):
        skymap, _ = MK.aux_variable(mm, model.unfold(binned), skymap, int(g["drv_ngibbs"]), draws)
        binned = RE.cls_centered(model, skymap)
        for sp in ("EE", "BB"):
            hist[sp].append(binned[sp])
    for sp in ("EE", "BB"):
        _close(np.array(hist[sp]), g["drv_h_" + sp])


def test_f1_pcg_fluctuations(g):
    """the PCG right-hand-side fluctuations match what the reference hands
    qcinv (captured by tools/gen_golden_masked.py), same numpy draws."""
    mm = _mm(g)
    np.random.seed(int(g["pcg_seed"]))
    d = MK.ReplayDraws()
    zp = d.pixel_normals(2, mm.Npix)
    zs = d.slot_normals(2, (mm.L + 1) ** 2)
    bf = MK.pcg_fluctuation(mm, _dl(g), zp, zs)
    _close(bf[0], g["pcg_bfluct_E"])
    _close(bf[1], g["pcg_bfluct_B"])


def test_f1_pcg_solves_the_system(g):
    mm = _mm(g)
    rng = np.random.default_rng(1)
    rhs = rng.standard_normal((2, (mm.L + 1) ** 2)) * 10
    rhs[:, mm.slot_ell < 2] = 0.0        # spin-2: Q is singular on l < 2 (no prior, no data)
    x, it = MK.pcg_solve(mm, _dl(g), rhs, tol=1e-12)
    res = MK.pcg_operator(mm, _dl(g), x) - rhs
    assert np.abs(res).max() < 1e-9 * np.abs(rhs).max()
    assert it < 500


def test_f2_pixel_likelihood_and_mh(g):
    """pixel-domain NC likelihood and one MH sweep (all_sph=False, masked)
    against the reference (tools/gen_golden_masked.py, seed f2_seed)."""
    mm = _mm(g)
    L = int(g["L"])
    bins = {"EE": g["bins_EE"], "BB": g["bins_BB"]}
    model = H.Model(L, int(g["nside"]), 2, g["bl"], [1.0, 1.0], bins,
                    blocks={"EE": g["blocks_EE"], "BB": g["blocks_BB"]},
                    proposal_variances={"EE": g["pv_EE"], "BB": g["pv_BB"]})
    snc = np.stack([g["f2_snc_E"], g["f2_snc_B"]])
    d_old = {"EE": g["init_EE"].copy(), "BB": g["init_BB"].copy()}
    lik0 = MK.nc_loglik_pixel(mm, model.unfold(d_old), snc)
    assert lik0 == pytest.approx(float(g["f2_lik0"]), rel=1e-11)
    np.random.seed(int(g["f2_seed"]))
    u_prop, u_acc = RE.draw_mh_uniforms(model)
    new, acc = MK.pixel_mh(mm, model, d_old, snc, u_prop=u_prop, u_accept=u_acc)
    _close(new["EE"], g["f2_EE"])
    _close(new["BB"], g["f2_BB"])
    assert acc["EE"] == list(g["f2_acc_EE"]) and acc["BB"] == list(g["f2_acc_BB"])


def test_f2_noncentre_roundtrip_and_chain_runs(g):
    mm = _mm(g)
    L = int(g["L"])
    bins = {"EE": g["bins_EE"], "BB": g["bins_BB"]}
    model = H.Model(L, int(g["nside"]), 2, g["bl"], [1.0, 1.0], bins,
                    blocks={"EE": g["blocks_EE"], "BB": g["blocks_BB"]},
                    proposal_variances={"EE": g["pv_EE"], "BB": g["pv_BB"]}, d_alm=np.zeros((2, (L + 1) ** 2)))
    dl = model.unfold({"EE": g["init_EE"], "BB": g["init_BB"]})
    s = _s_old(g)
    back = MK.noncentre(mm, dl, MK.noncentre(mm, dl, s), inverse=False)
    keep = mm.slot_ell >= 2
    _close(back[:, keep], s[:, keep])
    np.random.seed(5)
    h, acc, _ = MK.run_masked_mh_chain("noncentered", mm, model, {"EE": g["init_EE"], "BB": g["init_BB"]}, 1,
                                       MK.ReplayDraws(), tol=1e-10)
    assert h["EE"].shape == (2, len(g["init_EE"])) and np.all(np.isfinite(h["EE"]))
    assert acc["EE"].shape == (1, len(g["blocks_EE"]) - 1)
