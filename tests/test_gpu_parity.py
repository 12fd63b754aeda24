"""HIP path (through the C-ABI) vs the CPU oracle and the reference goldens.

Tolerances (fp64 everywhere):
  * layout / expansion helpers: exact or 1e-15 relative;
  * replay mode vs reference goldens: 1e-9 relative on D_l histories
    (north_star bar: 1e-6 relative on sampled C_l);
  * native mode vs oracle (same Philox streams): 1e-10 relative (libm ulps
    in log/sincos only).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import harmonic as H  # noqa: E402
from oracle import reference_eb as R  # noqa: E402
from tests._golden import load, model_from, init_of  # noqa: E402
from tests._util import stats_rows, rows_to_stats, make_problem  # noqa: E402

pytestmark = pytest.mark.gpu

SEED = 0x1234_5678_9ABC


def _plan(model, nchains=1, chain0=0, quirks=1, n_iter_metropolis=1):
    from gibbssampler_amd.engine import GibbsPlan
    return GibbsPlan(model.L, model.nside, model.nfields, nchains, model.bl, model.noise_var, model.bins,
                     blocks=model.blocks, proposal_variances=model.proposal_variances, chain0=chain0,
                     quirks=quirks, n_iter_metropolis=n_iter_metropolis)


def _dev(x):
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float64)).cuda()


@pytest.fixture(scope="module")
def g():
    return load(16)


# ---- stand-alone helpers ---------------------------------------------------------
def test_layout_helpers(g):
    from gibbssampler_amd import _capi as C
    lib = C.load()
    L = 37
    rng = np.random.RandomState(3)
    dl = rng.uniform(0, 5, size=(3, L + 1))
    var = torch.zeros(3, (L + 1) ** 2, dtype=torch.float64, device="cuda")
    C.check(lib.gs_var_expand(L, 3, C.ptr(_dev(dl)), C.ptr(var), C.stream_ptr()))
    np.testing.assert_allclose(var.cpu().numpy(), H.generate_var_cl(dl), rtol=1e-15, atol=0)
    x = rng.normal(size=(2, (L + 1) ** 2))
    cx = torch.zeros(2, (L + 1) * (L + 2), dtype=torch.float64, device="cuda")
    C.check(lib.gs_real_to_complex(L, 2, C.ptr(_dev(x)), C.ptr(cx), C.stream_ptr()))
    ref = np.stack([H.real_to_complex(x[k], L) for k in range(2)])
    got = cx.cpu().numpy().reshape(2, -1, 2)
    np.testing.assert_allclose(got[..., 0], ref.real, rtol=1e-15, atol=1e-300)
    np.testing.assert_allclose(got[..., 1], ref.imag, rtol=1e-15, atol=1e-300)
    back = torch.zeros(2, (L + 1) ** 2, dtype=torch.float64, device="cuda")
    C.check(lib.gs_complex_to_real(L, 2, C.ptr(cx), C.ptr(back), C.stream_ptr()))
    np.testing.assert_allclose(back.cpu().numpy(), np.stack([H.complex_to_real(r, L) for r in ref]), rtol=1e-15)
    y = _dev(x)
    C.check(lib.gs_remove_monopole_dipole(L, 2, C.ptr(y), C.stream_ptr()))
    np.testing.assert_array_equal(y.cpu().numpy(), np.stack([H.remove_monopole_dipole(r, L) for r in x]))
    cl = torch.zeros(2, L + 1, dtype=torch.float64, device="cuda")
    C.check(lib.gs_alm2cl(L, 2, C.ptr(_dev(x)), None, C.ptr(cl), C.stream_ptr()))
    np.testing.assert_allclose(cl.cpu().numpy(), np.stack([H.alm2cl_real(r) for r in x]), rtol=1e-13)
    # golden var expansion (reference generate_var_cl)
    gv = torch.zeros(1, (16 + 1) ** 2, dtype=torch.float64, device="cuda")
    C.check(lib.gs_var_expand(16, 1, C.ptr(_dev(g["a1_dl"][None])), C.ptr(gv), C.stream_ptr()))
    np.testing.assert_allclose(gv.cpu().numpy()[0], g["a1_var"], rtol=1e-15)


# ---- replay mode vs reference goldens -----------------------------------------------
def test_replay_centered_cr_a7(g):
    m = model_from(g)
    p = _plan(m)
    dl = p.dl_tensor({"EE": g["dl_EE"], "BB": g["dl_BB"]})   # unbinned EE bins; BB binned below
    dl_un = {"EE": g["dl_EE"], "BB": g["dl_BB"]}
    # the golden a7 uses unbinned spectra for both pols: use an unbinned plan
    m2 = model_from(g)
    m2.bins = {"EE": np.arange(m.L + 2), "BB": np.arange(m.L + 2)}
    m2.blocks = None
    m2.proposal_variances = None
    p = _plan(m2)
    dl = p.dl_tensor(dl_un)
    np.random.seed(int(g["a7_seed"]))
    z = p.replay_cr_normals()
    params = p.block_params(0, dl)
    s, _ = p.cr_sweep(p.data_tensor(m.d_alm), params, z=z)
    s = s.cpu().numpy()[0]
    np.testing.assert_allclose(s[0], g["a7_E"], rtol=1e-12, atol=1e-13)
    np.testing.assert_allclose(s[1], g["a7_B"], rtol=1e-12, atol=1e-13)


def test_replay_noncentered_cr_a8(g):
    m = model_from(g)
    m.bins = {"EE": np.arange(m.L + 2), "BB": np.arange(m.L + 2)}
    m.blocks = m.proposal_variances = None
    p = _plan(m)
    dl = p.dl_tensor({"EE": g["dl_EE"], "BB": g["dl_BB"]})
    np.random.seed(int(g["a8_seed"]))
    s, _ = p.cr_sweep(p.data_tensor(m.d_alm), p.block_params(1, dl), z=p.replay_cr_normals())
    s = s.cpu().numpy()[0]
    np.testing.assert_allclose(s[0], g["a8_E"], rtol=1e-12, atol=1e-13)
    np.testing.assert_allclose(s[1], g["a8_B"], rtol=1e-12, atol=1e-13)


def test_replay_centered_cls_a13(g):
    m = model_from(g)
    p = _plan(m)
    s = np.stack([g["a7_E"], g["a7_B"]])
    stats = _dev(stats_rows(2, H.sweep_stats(m, s, m.d_alm))[None])
    np.random.seed(int(g["a13_seed"]))
    out = p.dl_dicts(p.cls_draw(stats, variates=p.replay_invgamma()))[0]
    np.testing.assert_allclose(out["EE"], g["a13_EE"], rtol=1e-10)
    np.testing.assert_allclose(out["BB"], g["a13_BB"], rtol=1e-10)


def test_replay_nc_mh_a15(g):
    m = model_from(g)
    p = _plan(m)
    s = np.stack([g["a8_E"], g["a8_B"]])
    stats = _dev(stats_rows(2, H.sweep_stats(m, s, m.d_alm))[None])
    np.random.seed(int(g["a15_seed"]))
    up, ua = p.replay_mh_uniforms()
    dl = p.dl_tensor(init_of(g))
    acc = p.split_accept(p.nc_mh(stats, dl, up, ua))
    out = p.dl_dicts(dl)[0]
    np.testing.assert_array_equal(acc["EE"][0], g["a15_acc_EE"])
    np.testing.assert_array_equal(acc["BB"][0], g["a15_acc_BB"])
    np.testing.assert_allclose(out["EE"], g["a15_EE"], rtol=1e-9)
    np.testing.assert_allclose(out["BB"], g["a15_BB"], rtol=1e-9)


def test_replay_drivers_match_reference(g):
    """Full NonCenteredGibbs / CenteredGibbs / ASIS runs (replay) == reference."""
    from gibbssampler_amd import samplers
    m = model_from(g)
    common = dict(lmax=m.L, nside=m.nside, bl=m.bl, noise_var=m.noise_var, bins=m.bins, blocks=m.blocks,
                  proposal_variances=m.proposal_variances, d_alm={"EE": g["d_E"], "BB": g["d_B"]})
    for kind, seed, key in (("noncentered", "nc_seed", "nc_h"), ("centered", "c_seed", "c_h"),
                            ("asis", "asis_seed", "asis_h")):
        run = samplers.BatchedRunner(kind=kind, nfields=2, nchains=1, rng="replay", **common)
        np.random.seed(int(g[seed]))
        h, acc = run.run(init_of(g), int(g[key.split("_")[0] + "_iters"]))
        np.testing.assert_allclose(h["EE"][:, 0], g[key + "_EE"], rtol=1e-9, err_msg=kind)
        np.testing.assert_allclose(h["BB"][:, 0], g[key + "_BB"], rtol=1e-9, err_msg=kind)


# ---- native mode vs oracle (same counter streams) ---------------------------------------
@pytest.mark.parametrize("F", [1, 2, 3])
@pytest.mark.parametrize("mode", [0, 1])
def test_native_cr_sweep_matches_oracle(F, mode):
    L, nside = 45, 16
    m, init = make_problem(L, nside, F, seed=11)
    nch, chain0, it = 3, 5, 7
    p = _plan(m, nchains=nch, chain0=chain0)
    dl = p.dl_tensor(init)
    params = p.block_params(mode, dl)
    s, st = p.cr_sweep(p.data_tensor(m.d_alm), params, seed=SEED, iteration=it, substep=0)
    s, st = s.cpu().numpy(), st.cpu().numpy()
    un = m.unfold(init)
    M, Lc = (H.centered_params if mode == 0 else H.noncentered_params)(m, un)
    np.testing.assert_allclose(params.cpu().numpy()[0, :, :1], M[:, :1, 0], rtol=1e-12)
    for c in range(nch):
        z = np.stack([H.cr_normals(SEED, chain0 + c, it, 0, f, L) for f in range(F)])
        ref = H.cr_apply(m, M, Lc, m.d_alm, z)
        np.testing.assert_allclose(s[c], ref, rtol=1e-10, atol=1e-12 * np.abs(ref).max())
        rows = stats_rows(F, H.sweep_stats(m, ref, m.d_alm))
        np.testing.assert_allclose(st[c], rows, rtol=1e-10, atol=1e-12 * np.abs(rows).max())


@pytest.mark.parametrize("F", [1, 2, 3])
def test_native_cls_draw_matches_oracle(F):
    L, nside = 40, 16
    m, init = make_problem(L, nside, F, seed=5)
    p = _plan(m, nchains=2, chain0=3)
    rng = np.random.RandomState(9)
    dl = p.dl_tensor(init)
    s, st = p.cr_sweep(p.data_tensor(m.d_alm), p.block_params(0, dl), seed=SEED, iteration=2)
    out = p.dl_dicts(p.cls_draw(st, seed=SEED, iteration=2))
    stn = st.cpu().numpy()
    for c in range(2):
        ref = H.centered_cls_draw(m, rows_to_stats(F, stn[c]), seed=SEED, chain=3 + c, iteration=2)
        for sp in m.spectra:
            np.testing.assert_allclose(out[c][sp], ref[sp], rtol=1e-10, err_msg=sp)
    del rng


@pytest.mark.parametrize("F", [1, 2, 3])
@pytest.mark.parametrize("n_iter", [1, 2])
def test_native_nc_mh_matches_oracle(F, n_iter):
    L, nside = 40, 16
    m, init = make_problem(L, nside, F, seed=6)
    p = _plan(m, nchains=2, chain0=1, n_iter_metropolis=n_iter)
    dl = p.dl_tensor(init)
    _, st = p.cr_sweep(p.data_tensor(m.d_alm), p.block_params(1, dl), seed=SEED, iteration=4)
    acc = p.split_accept(p.nc_mh(st, dl, seed=SEED, iteration=4))
    out = p.dl_dicts(dl)
    stn = st.cpu().numpy()
    for c in range(2):
        ref, racc = H.nc_mh(m, init, rows_to_stats(F, stn[c]), seed=SEED, chain=1 + c, iteration=4,
                            n_iter=n_iter)
        for sp in m.spectra:
            np.testing.assert_array_equal(acc[sp][c], np.array(racc[sp]), err_msg=sp)
            np.testing.assert_allclose(out[c][sp], ref[sp], rtol=1e-10, err_msg=sp)


def test_native_stats_to_noncentered_and_recentre():
    L, nside, F = 30, 16, 3
    m, init = make_problem(L, nside, F, seed=2)
    p = _plan(m, nchains=1)
    dl = p.dl_tensor(init)
    s, st = p.cr_sweep(p.data_tensor(m.d_alm), p.block_params(0, dl), seed=SEED, iteration=1)
    ref_st = rows_to_stats(F, st.cpu().numpy()[0])
    A = H.cov_chol(m, m.unfold(init))
    T = H.chol_pinv(A)
    exp = stats_rows(F, H.transform_stats(ref_st, T))
    got = p.stats_to_noncentered(dl, st).cpu().numpy()[0]
    np.testing.assert_allclose(got, exp, rtol=1e-10, atol=1e-12 * np.abs(exp).max())
    # recentre: s <- A s
    s0 = s.cpu().numpy()[0]
    p.recentre(dl, s)
    ell = H.slot_ell(L)
    ref = np.einsum("sfg,gs->fs", A[ell], s0)
    np.testing.assert_allclose(s.cpu().numpy()[0], ref, rtol=1e-12, atol=1e-14 * np.abs(ref).max())
