"""GPU: the masked CR samplers (gs_masked_cr through gibbssampler_amd.masked.MaskedCR).

Replay mode against the reference-generated fixtures (same numpy draws, same
algebra: a9 aux-variable, a10 over-relaxation, a11 MALA incl. both accept
branches, a12 composition) and native mode against the oracle's restatement
of the device Philox streams (EB and the TEB generalisation)."""
import os

import numpy as np
import pytest

from oracle import masked as MK
from oracle import sht as O

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_masked_eb_N8_L16.npz")
TOL = dict(rtol=1e-9)


@pytest.fixture(scope="module")
def g():
    return dict(np.load(GOLDEN))


def _cr(g, **kw):
    from gibbssampler_amd.masked import MaskedCR
    pix = {"Q": g["Q"], "U": g["U"]}
    return MaskedCR(pix, 40.0 ** 2, g["noise_pol"], g["bl"], int(g["L"]), int(g["nside"]), mask=g["mask"], **kw)


def _dls(g):
    return {"EE": g["dl_EE"], "BB": g["dl_BB"]}


def _sold(g):
    return {"EE": g["s_old_E"].copy(), "BB": g["s_old_B"].copy()}


def _close(got, want):
    np.testing.assert_allclose(got, want, rtol=1e-9, atol=1e-11 * np.abs(want).max())


def test_constants(g):
    cr = _cr(g)
    assert cr.mu[1] == pytest.approx(float(g["mu"]), rel=1e-15)
    g2 = cr.second_part_grad().cpu().numpy()
    _close(g2[0], g["second_part_grad_E"])
    _close(g2[1], g["second_part_grad_B"])


def test_a9_replay(g):
    cr = _cr(g, n_gibbs=int(g["a9_ngibbs"]))
    np.random.seed(int(g["a9_seed"]))
    s, acc = cr.sample_gibbs_change_variable(_dls(g), _sold(g))
    assert acc == 1
    _close(s["EE"], g["a9_E"])
    _close(s["BB"], g["a9_B"])


def test_a10_replay(g):
    cr = _cr(g, n_gibbs=int(g["a10_ngibbs"]), overrelaxation=True, alpha=float(g["a10_alpha"]))
    np.random.seed(int(g["a10_seed"]))
    s, acc = cr.overrelaxation_sampler(_dls(g), _sold(g))
    assert acc == 1
    _close(s["EE"], g["a10_E"])
    _close(s["BB"], g["a10_B"])


def test_a11_gradient(g):
    cr = _cr(g, gibbs_cr=False, ula=True)
    gE, gB, pE, pB = cr.compute_gradient_mala(_dls(g), _sold(g))
    _close(gE, g["a11_gradE"])
    _close(gB, g["a11_gradB"])
    _close(pE, g["a11_sEpix"])
    _close(pB, g["a11_sBpix"])


@pytest.mark.parametrize("variant", ["a11", "a11b"])
def test_a11_mala_replay(g, variant):
    tau = float(g["a11_tau"]) if variant == "a11" else float(g["a11b_tau"])
    cr = _cr(g, gibbs_cr=False, ula=True, tau=tau)
    start = _sold(g) if variant == "a11" else {"EE": g["a9_E"], "BB": g["a9_B"]}
    for k, sd in enumerate(g[variant + "_seeds"]):
        np.random.seed(int(sd))
        s, acc = cr.sample_mala(_dls(g), start)
        assert acc == int(g[variant + "_accept"][k])
        _close(s["EE"], g[variant + "_E"][k])
        _close(s["BB"], g[variant + "_B"][k])


def test_a12_composition_replay(g):
    cr = _cr(g, gibbs_cr=True, ula=True, n_gibbs=int(g["a12_ngibbs"]))
    np.random.seed(int(g["a12_seed"]))
    s, acc = cr.sample(_dls(g), _sold(g))
    assert acc == int(g["a12_accept"])
    _close(s["EE"], g["a12_E"])
    _close(s["BB"], g["a12_B"])


def _teb_problem(N=8, L=16, seed=3):
    rng = np.random.default_rng(seed)
    npix = 12 * N * N
    th, _ = O.pixel_angles(N)
    mask = (np.abs(np.cos(th)) > 0.2).astype(float)
    maps = rng.standard_normal((3, npix)) * np.array([[30.0], [0.3], [0.3]])
    ntemp = np.full(npix, 40.0 ** 2) * np.linspace(0.9, 1.1, npix)
    npol = np.full(npix, 0.2 ** 2) * np.linspace(1.2, 0.8, npix)
    ell = np.arange(L + 1)
    bl = np.exp(-0.5 * ell * (ell + 1) * (0.07 / np.sqrt(8 * np.log(2))) ** 2)
    dl = {"TT": np.where(ell >= 2, 1000.0, 0.0), "EE": np.where(ell >= 2, 10.0 * (np.maximum(ell, 1) / 100) ** 0.5, 0),
          "BB": np.where(ell >= 2, 0.01, 0.0)}
    dl["TE"] = 0.5 * np.sqrt(dl["TT"] * dl["EE"])
    s0 = rng.standard_normal((3, (L + 1) ** 2)) * np.array([[3.0], [0.05], [0.005]])
    return N, L, mask, maps, ntemp, npol, bl, dl, s0


@pytest.mark.parametrize("F", [2, 3])
@pytest.mark.parametrize("over", [False, True])
def test_aux_native_vs_oracle(F, over):
    from gibbssampler_amd.masked import MaskedCR
    N, L, mask, maps, ntemp, npol, bl, dl, s0 = _teb_problem()
    seed, it, chain, ng = 4242, 7, 3, 2
    pix = {"T": maps[0], "Q": maps[1], "U": maps[2]}
    cr = MaskedCR(pix, ntemp, npol, bl, L, N, mask=mask, nfields=F, n_gibbs=ng, overrelaxation=over, rng="native",
                  seed=seed, chain=chain)
    cr.iteration = it
    rows = (1, 2) if F == 2 else (0, 1, 2)
    fields = ("EE", "BB") if F == 2 else ("TT", "EE", "BB")
    s_in = {k: s0[r] for k, r in zip(fields, rows)}
    s, acc = (cr.overrelaxation_sampler if over else cr.sample_gibbs_change_variable)(dl, s_in)
    inv = np.stack([mask / ntemp, mask / npol, mask / npol])
    mm = MK.MaskedModel(L, N, F, bl, maps, inv)
    spec = ("EE", "BB") if F == 2 else ("TT", "EE", "BB", "TE")
    dlu = np.stack([dl[k] for k in spec])
    draws = MK.NativeDraws(seed, chain, it, L, 12 * N * N)
    start = np.stack([s0[r] for r in rows])
    if over:
        want, _ = MK.overrelaxation(mm, dlu, start, ng, draws)
    else:
        want, _ = MK.aux_variable(mm, dlu, start, ng, draws)
    for k, f in enumerate(fields):
        _close(s[f], want[k])


def test_mala_native_vs_oracle():
    from gibbssampler_amd.masked import MaskedCR
    N, L, mask, maps, ntemp, npol, bl, dl, s0 = _teb_problem(seed=5)
    seed, it, chain = 99, 4, 1
    for tau in (1e-4, 0.6):
        cr = MaskedCR({"Q": maps[1], "U": maps[2]}, ntemp, npol, bl, L, N, mask=mask, nfields=2, gibbs_cr=False,
                      ula=True, tau=tau, rng="native", seed=seed, chain=chain)
        cr.iteration = it
        s, acc = cr.sample_mala(dl, {"EE": s0[1], "BB": s0[2]})
        mm = MK.MaskedModel(L, N, 2, bl, maps, np.stack([mask / ntemp, mask / npol, mask / npol]))
        want, wacc, lr = MK.mala(mm, np.stack([dl["EE"], dl["BB"]]), s0[1:], MK.NativeDraws(seed, chain, it, L, 12 * N * N),
                                 float(npol[0]), tau=tau)
        assert acc == wacc
        np.testing.assert_allclose(cr.last_log_ratio(), lr, rtol=1e-8, atol=1e-8)
        _close(s["EE"], want[0])
        _close(s["BB"], want[1])


def test_masked_centered_driver_replay(g):
    """CenteredGibbs(mask_path=..., gibbs_cr=True) end to end on the device:
    GibbsSampler.run_polarization with the a9 CR and the invgamma C_l draw,
    against the reference driver (start map injected for the qcinv init)."""
    from gibbssampler_amd.gibbs import CenteredGibbs
    L, N = int(g["L"]), int(g["nside"])
    cg = CenteredGibbs({"Q": g["Q"], "U": g["U"]}, np.full(12 * N * N, 40.0 ** 2), g["noise_pol"],
                       float(g["fwhm_deg"]), N, L, 12 * N * N, mask_path=g["mask"], polarization=True,
                       bins={"EE": g["bins_EE"], "BB": g["bins_BB"]}, n_iter=int(g["drv_iters"]), gibbs_cr=True,
                       overrelaxation=False, ula=False, rng="replay", n_gibbs=int(g["drv_ngibbs"]),
                       skymap_init={"EE": g["s_old_E"], "BB": g["s_old_B"]})
    np.random.seed(int(g["drv_seed"]))
    h, acc, tcr, tcls = cg.run({"EE": g["init_EE"].copy(), "BB": g["init_BB"].copy()})
    assert np.all(acc == 1)
    _close(h["EE"], g["drv_h_EE"])
    _close(h["BB"], g["drv_h_BB"])


def test_masked_teb_driver_native_runs():
    """TEB masked run (native streams): finite, positive-definite draws."""
    from gibbssampler_amd.gibbs import CenteredGibbs
    N, L, mask, maps, ntemp, npol, bl, dl, s0 = _teb_problem()
    cg = CenteredGibbs({"T": maps[0], "Q": maps[1], "U": maps[2]}, ntemp, npol, 4.0, N, L, 12 * N * N,
                       mask_path=mask, polarization=True, fields="TEB", n_iter=4, gibbs_cr=True, rng="native",
                       seed=11, n_gibbs=2)
    init = {"TT": dl["TT"][:L + 1], "EE": dl["EE"][:L + 1], "BB": dl["BB"][:L + 1], "TE": dl["TE"][:L + 1]}
    h, acc, _, _ = cg.run(init)
    for s in ("TT", "EE", "BB", "TE"):
        assert h[s].shape == (5, L + 1) and np.all(np.isfinite(h[s]))
    assert np.all(h["TT"][1:, 2:] > 0) and np.all(h["EE"][1:, 2:] > 0) and np.all(h["BB"][1:, 2:] > 0)
    assert np.all(h["TE"][1:, 2:] ** 2 < h["TT"][1:, 2:] * h["EE"][1:, 2:])


# ---- f1: PCG constrained realisation --------------------------------------------------
def _dl_t(cr, d):
    import torch
    return torch.from_numpy(np.ascontiguousarray(np.stack([d["EE"], d["BB"]]))).cuda()


def test_f1_pcg_rhs_replay(g):
    """the right-hand side the device builds = the reference's b_fluctuations
    (captured from its qcinv call) + b A^T N^-1 d, same numpy draws."""
    cr = _cr(g, gibbs_cr=False, ula=False)
    np.random.seed(int(g["pcg_seed"]))
    rhs = cr.pcg_rhs(_dl_t(cr, _dls(g))).cpu().numpy()
    g2 = cr.second_part_grad().cpu().numpy()
    _close(rhs[0] - g2[0], g["pcg_bfluct_E"])
    _close(rhs[1] - g2[1], g["pcg_bfluct_B"])


def test_f1_pcg_solve_vs_oracle(g):
    import torch
    cr = _cr(g, gibbs_cr=False, ula=False)
    mm = MK.MaskedModel(int(g["L"]), int(g["nside"]), 2, g["bl"],
                        np.stack([np.zeros(768), g["Q"], g["U"]]),
                        np.stack([np.zeros(768), g["inv_noise_pol"], g["inv_noise_pol"]]))
    rng = np.random.default_rng(3)
    rhs = rng.standard_normal((2, mm.NR if hasattr(mm, "NR") else (mm.L + 1) ** 2)) * 10
    rhs[:, mm.slot_ell < 2] = 0.0
    dl = np.stack([g["dl_EE"], g["dl_BB"]])
    want, _ = MK.pcg_solve(mm, dl, rhs, tol=1e-13)
    x = cr.pcg_solve(torch.from_numpy(dl).cuda(), torch.from_numpy(rhs).cuda(), tol=1e-13).cpu().numpy()
    assert cr.pcg_residual <= 1e-13
    _close(x, want)


@pytest.mark.parametrize("F", [2, 3])
def test_f1_pcg_sample_native_vs_oracle(F):
    from gibbssampler_amd.masked import MaskedCR
    N, L, mask, maps, ntemp, npol, bl, dl, s0 = _teb_problem(seed=7)
    seed, it, chain = 31, 2, 5
    cr = MaskedCR({"T": maps[0], "Q": maps[1], "U": maps[2]}, ntemp, npol, bl, L, N, mask=mask, nfields=F,
                  gibbs_cr=False, ula=False, rng="native", seed=seed, chain=chain, pcg_accuracy=1e-13)
    cr.iteration = it
    s, acc = cr.sample_mask(dl)
    assert acc == 1 and cr.pcg_residual <= 1e-13
    mm = MK.MaskedModel(L, N, F, bl, maps, np.stack([mask / ntemp, mask / npol, mask / npol]))
    spec = ("EE", "BB") if F == 2 else ("TT", "EE", "BB", "TE")
    want, _, _ = MK.pcg_sample(mm, np.stack([dl[k] for k in spec]), MK.NativeDraws(seed, chain, it, L, 12 * N * N),
                               tol=1e-13)
    fields = ("EE", "BB") if F == 2 else ("TT", "EE", "BB")
    for k, f in enumerate(fields):
        _close(s[f], want[k])


@pytest.mark.parametrize("F,rng", [(2, "native"), (3, "native"), (2, "replay")])
def test_rj_sample_vs_oracle(F, rng):
    """sample_mask_rj (CenteredGibbs.py:606-674) against the oracle restatement
    (oracle/masked.py: rj_sample; the reference's RJPO needs qcinv, absent here,
    so this row is pinned by the oracle only): the PCG started from -s_old and
    cut at 6 iterations (tol 0), so the log ratio -sum (rhs - Q x).(s_old - x)
    is macroscopic; the map, the log ratio and the decision agree."""
    import torch
    from gibbssampler_amd.masked import MaskedCR
    N, L, mask, maps, ntemp, npol, bl, dl, s0 = _teb_problem(seed=11)
    seed, it, chain = 77, 3, 1
    cr = MaskedCR({"T": maps[0], "Q": maps[1], "U": maps[2]}, ntemp, npol, bl, L, N, mask=mask, nfields=F,
                  gibbs_cr=False, ula=False, rng=rng, seed=seed, chain=chain, pcg_accuracy=0.0, pcg_maxiter=6, rj=True)
    cr.iteration = it
    rows = (1, 2) if F == 2 else (0, 1, 2)
    fields = ("EE", "BB") if F == 2 else ("TT", "EE", "BB")
    s_in = {k: s0[r] for k, r in zip(fields, rows)}
    if rng == "replay":
        np.random.seed(5)
    s, acc = cr.sample(dl, s_in)                # the ladder's RJ branch (rj=True)
    assert cr.pcg_iterations[-1] == 6
    mm = MK.MaskedModel(L, N, F, bl, maps, np.stack([mask / ntemp, mask / npol, mask / npol]))
    spec = ("EE", "BB") if F == 2 else ("TT", "EE", "BB", "TE")
    draws = MK.NativeDraws(seed, chain, it, L, 12 * N * N) if rng == "native" else MK.ReplayDraws(5)
    want, wacc, lp, wit = MK.rj_sample(mm, np.stack([dl[k] for k in spec]), draws, np.stack([s0[r] for r in rows]),
                                       tol=0.0, maxiter=6)
    assert wit == 6
    assert abs(cr.last_log_ratio() - lp) <= 1e-8 * max(1.0, abs(lp))
    assert acc == wacc
    for k, f in enumerate(fields):
        _close(s[f], want[k])
    # the same step through the runner kind (device state in place, no host copy)
    s_t = torch.from_numpy(np.ascontiguousarray(np.stack([s0[r] for r in rows]))).cuda()
    dl_t = torch.from_numpy(np.ascontiguousarray(np.stack([dl[k] for k in spec]))).cuda()
    if rng == "replay":
        np.random.seed(5)
    cr.rj_step(dl_t, s_t, iteration=it)
    np.testing.assert_array_equal(s_t.cpu().numpy(), np.stack([s[f] for f in fields]))


def test_f1_pcg_driver_replay_vs_oracle(g):
    """CenteredGibbs(mask, gibbs_cr=False, ula=False): PCG init CR + PCG CR +
    invgamma draws (HEAD's default masked path) against the oracle chain."""
    from gibbssampler_amd.gibbs import CenteredGibbs
    L, N = int(g["L"]), int(g["nside"])
    bins = {"EE": g["bins_EE"], "BB": g["bins_BB"]}
    cg = CenteredGibbs({"Q": g["Q"], "U": g["U"]}, np.full(12 * N * N, 40.0 ** 2), g["noise_pol"],
                       float(g["fwhm_deg"]), N, L, 12 * N * N, mask_path=g["mask"], polarization=True, bins=bins,
                       n_iter=3, gibbs_cr=False, ula=False, rng="replay")
    cg.constrained_sampler.pcg_accuracy = 1e-13
    np.random.seed(2024)
    h, acc, _, _ = cg.run({"EE": g["init_EE"].copy(), "BB": g["init_BB"].copy()})
    # oracle chain, same draw order: PCG init, then per iteration PCG + invgamma EE, BB
    from oracle import harmonic as H
    from oracle import reference_eb as RE
    mm = MK.MaskedModel(L, N, 2, g["bl"], np.stack([np.zeros(768), g["Q"], g["U"]]),
                        np.stack([np.zeros(768), g["inv_noise_pol"], g["inv_noise_pol"]]))
    model = H.Model(L, N, 2, g["bl"], [1.0, 1.0], bins, d_alm=np.zeros((2, (L + 1) ** 2)))
    np.random.seed(2024)
    binned = {"EE": g["init_EE"].copy(), "BB": g["init_BB"].copy()}
    draws = MK.ReplayDraws()
    MK.pcg_sample(mm, model.unfold(binned), draws, tol=1e-13)
    want = {"EE": [binned["EE"]], "BB": [binned["BB"]]}
    for _ in range(3):
        s, _, _ = MK.pcg_sample(mm, model.unfold(binned), draws, tol=1e-13)
        binned = RE.cls_centered(model, s)
        for sp in ("EE", "BB"):
            want[sp].append(binned[sp])
    assert np.all(acc == 1)
    for sp in ("EE", "BB"):
        np.testing.assert_allclose(h[sp], np.array(want[sp]), rtol=1e-7)


# ---- f2: pixel-domain non-centred likelihood --------------------------------------------
def _f2_parts(g):
    bins = {"EE": g["bins_EE"], "BB": g["bins_BB"]}
    blocks = {"EE": g["blocks_EE"], "BB": g["blocks_BB"]}
    pv = {"EE": g["pv_EE"], "BB": g["pv_BB"]}
    return bins, blocks, pv


def _oracle_model(g):
    from oracle import harmonic as H
    L, N = int(g["L"]), int(g["nside"])
    bins, blocks, pv = _f2_parts(g)
    mm = MK.MaskedModel(L, N, 2, g["bl"], np.stack([np.zeros(768), g["Q"], g["U"]]),
                        np.stack([np.zeros(768), g["inv_noise_pol"], g["inv_noise_pol"]]))
    model = H.Model(L, N, 2, g["bl"], [1.0, 1.0], bins, blocks=blocks, proposal_variances=pv,
                    d_alm=np.zeros((2, (L + 1) ** 2)))
    return mm, model


def test_f2_pixel_mh_replay(g):
    """the device likelihood and one MH sweep = the reference's
    PolarizationNonCenteredClsSampler.sample(all_sph=False) (fixture f2_*)."""
    from gibbssampler_amd.masked import PixelMH
    bins, blocks, pv = _f2_parts(g)
    mh = PixelMH(_cr(g, gibbs_cr=False, ula=False), bins, blocks, pv)
    snc = {"EE": g["f2_snc_E"], "BB": g["f2_snc_B"]}
    init = {"EE": g["init_EE"].copy(), "BB": g["init_BB"].copy()}
    assert mh.compute_log_likelihood(init, snc) == pytest.approx(float(g["f2_lik0"]), rel=1e-11)
    np.random.seed(int(g["f2_seed"]))
    new, acc = mh.sample(snc, init)
    _close(new["EE"], g["f2_EE"])
    _close(new["BB"], g["f2_BB"])
    assert acc["EE"] == list(g["f2_acc_EE"]) and acc["BB"] == list(g["f2_acc_BB"])


def test_f2_pixel_mh_native_vs_oracle(g):
    from gibbssampler_amd.masked import PixelMH
    bins, blocks, pv = _f2_parts(g)
    seed, chain, it = 77, 3, 5
    cr = _cr(g, gibbs_cr=False, ula=False, rng="native", seed=seed, chain=chain)
    mh = PixelMH(cr, bins, blocks, pv)
    snc = np.stack([g["f2_snc_E"], g["f2_snc_B"]])
    init = {"EE": g["init_EE"].copy(), "BB": g["init_BB"].copy()}
    new, acc = mh.sample(snc, init, iteration=it)
    mm, model = _oracle_model(g)
    want, wacc = MK.pixel_mh(mm, model, init, snc, seed=seed, chain=chain, iteration=it)
    _close(new["EE"], want["EE"])
    _close(new["BB"], want["BB"])
    assert acc == wacc


def _masked_mh_sampler(g, cls, n_iter, rng="replay", seed=0, **kw):
    from gibbssampler_amd import gibbs as G
    L, N = int(g["L"]), int(g["nside"])
    bins, blocks, pv = _f2_parts(g)
    args = ({"Q": g["Q"], "U": g["U"]}, np.full(12 * N * N, 40.0 ** 2), g["noise_pol"], float(g["fwhm_deg"]), N, L,
            12 * N * N, pv)
    smp = getattr(G, cls)(*args, metropolis_blocks=blocks, polarization=True, bins=bins, n_iter=n_iter,
                          mask_path=g["mask"], rng=rng, seed=seed, **kw)
    smp.masked_cr.pcg_accuracy = 1e-13
    return smp


@pytest.mark.parametrize("rng", ["replay", "native"])
def test_f2_masked_noncentered_driver_vs_oracle(g, rng):
    """NonCenteredGibbs(mask_path=...): per iteration the PCG CR, C^-1/2, the
    pixel MH sweep (NonCenteredGibbs.py:529-571), against the oracle chain."""
    smp = _masked_mh_sampler(g, "NonCenteredGibbs", 3, rng=rng, seed=19)
    init = {"EE": g["init_EE"].copy(), "BB": g["init_BB"].copy()}
    np.random.seed(808)
    h, acc, _, _ = smp.run(init)
    mm, model = _oracle_model(g)
    np.random.seed(808)
    if rng == "replay":
        want, wacc, _ = MK.run_masked_mh_chain("noncentered", mm, model, init, 3, MK.ReplayDraws())
    else:
        want, wacc, _ = MK.run_masked_mh_chain("noncentered", mm, model, init, 3,
                                               lambda it: MK.NativeDraws(19, 0, it, mm.L, mm.Npix), native=(19, 0))
    for sp in ("EE", "BB"):
        np.testing.assert_allclose(h[sp], want[sp], rtol=1e-7)
        np.testing.assert_array_equal(acc[sp], wacc[sp])


@pytest.mark.parametrize("gibbs_cr", [False, True])
def test_f2_masked_asis_driver_vs_oracle(g, gibbs_cr):
    """ASIS(mask_path=...): CR (PCG, or the aux + MALA composition with its
    PCG start map), centred C_l draw, non-centring, pixel MH, re-centring with
    the reference's quirk (ASIS.py:134-226), against the oracle chain."""
    n_gibbs = 2
    smp = _masked_mh_sampler(g, "ASIS", 3, gibbs_cr=gibbs_cr, n_gibbs=n_gibbs)
    init = {"EE": g["init_EE"].copy(), "BB": g["init_BB"].copy()}
    np.random.seed(909)
    out = smp.run(init)
    h, acc = out[0], out[1]
    assert len(out) == 7
    mm, model = _oracle_model(g)
    np.random.seed(909)
    want, wacc, _ = MK.run_masked_mh_chain("asis", mm, model, init, 3, MK.ReplayDraws(),
                                           cr="aux_mala" if gibbs_cr else "pcg", n_gibbs=n_gibbs,
                                           noise_pol0=float(g["noise_pol"][0]))
    for sp in ("EE", "BB"):
        np.testing.assert_allclose(h[sp], want[sp], rtol=1e-7)
        np.testing.assert_array_equal(acc[sp], wacc[sp])


@pytest.mark.parametrize("n_iter,group_bytes,stage", [(1, None, "1"), (2, None, "1"), (2, "1", "1"),
                                                     (1, "50000000", "1"), (1, None, "0"), (2, "1", "0")])
def test_f2_device_sweep_groups_vs_oracle(g, monkeypatch, n_iter, group_bytes, stage):
    """gs_masked_pixel_mh decides every block on the device from one block
    synthesis + one Gram pass; with a small workspace budget the blocks run in
    groups (one block per group at "1") and the residual is carried between
    groups.  Native streams, n_iter_metropolis 1 and 2, against the oracle's
    full-map likelihood per block (oracle/masked.pixel_mh).  stage "0": the
    block synthesis without the LDS-staged inputs (the large-l_max form)."""
    from gibbssampler_amd.masked import PixelMH
    monkeypatch.setenv("GS_SHT_BLK_STAGE", stage)
    if group_bytes is not None:
        monkeypatch.setenv("GS_F2_GROUP_BYTES", group_bytes)
    bins, blocks, pv = _f2_parts(g)
    seed, chain, it = 313, 1, 9
    cr = _cr(g, gibbs_cr=False, ula=False, rng="native", seed=seed, chain=chain)
    mh = PixelMH(cr, bins, blocks, pv, n_iter_metropolis=n_iter)
    assert mh.K >= 3
    snc = np.stack([g["f2_snc_E"], g["f2_snc_B"]])
    init = {"EE": g["init_EE"].copy(), "BB": g["init_BB"].copy()}
    new, acc = mh.sample(snc, init, iteration=it)
    mm, model = _oracle_model(g)
    want, wacc = MK.pixel_mh(mm, model, init, snc, seed=seed, chain=chain, iteration=it, n_iter=n_iter)
    _close(new["EE"], want["EE"])
    _close(new["BB"], want["BB"])
    assert acc == wacc


@pytest.fixture(scope="module")
def f2_large():
    """N_side 32, l_max 70, unbinned EE and BB with one Metropolis block per bin
    from bin 2: 69 + 69 = 138 blocks, so one Gram group has R = 139 rows (G's
    triangle 77.8 KB: the > 64 KB dynamic-LDS decision path) and the Gram pass
    an uneven number of chunks."""
    from gibbssampler_amd.problem import gauss_beam
    N, L = 32, 70
    npix = 12 * N * N
    rng = np.random.default_rng(4242)
    theta, _ = O.pixel_angles(N)
    mask = (np.abs(np.cos(theta)) > 0.2).astype(np.float64)
    bins = {"EE": np.arange(0, L + 2), "BB": np.arange(0, L + 2)}
    blocks = {"EE": np.arange(2, L + 2), "BB": np.arange(2, L + 2)}
    dl = {"EE": np.r_[0.0, 0.0, 10.0 * (np.arange(2, L + 1) / 100.0) ** 0.5], "BB": np.r_[0.0, 0.0, np.full(L - 1, 0.05)]}
    pv = {"EE": (0.02 * dl["EE"][2:]) ** 2, "BB": np.full(L - 1, 0.01) ** 2}     # bins >= 2
    pix = {"Q": rng.normal(0, 0.5, npix), "U": rng.normal(0, 0.5, npix)}
    snc = rng.normal(size=(2, (L + 1) ** 2))
    return dict(N=N, L=L, mask=mask, bins=bins, blocks=blocks, dl=dl, pv=pv, pix=pix, snc=snc,
                bl=gauss_beam(np.radians(0.5), L))


@pytest.mark.parametrize("n_iter", [1, 20, 90])
def test_f2_large_group_decisions_equal_one_block_groups(f2_large, monkeypatch, n_iter):
    """the large-R decision path (138 blocks in one group, G's
    triangle beyond 64 KB of LDS) and n_iter_metropolis up to 90 (the log
    uniforms then no longer fit in LDS beside the triangle and are read from
    global memory) decide exactly as one block per group, whose path the
    small-fixture tests pin against the oracle's full-map likelihood."""
    from gibbssampler_amd.masked import MaskedCR, PixelMH
    q = f2_large
    out = []
    for group_bytes in (None, "1"):
        if group_bytes is None:
            monkeypatch.delenv("GS_F2_GROUP_BYTES", raising=False)
        else:
            monkeypatch.setenv("GS_F2_GROUP_BYTES", group_bytes)
        cr = MaskedCR(q["pix"], 40.0 ** 2, np.full(12 * q["N"] ** 2, 0.2 ** 2), q["bl"], q["L"], q["N"],
                      mask=q["mask"], gibbs_cr=False, ula=False, rng="native", seed=515, chain=2)
        mh = PixelMH(cr, q["bins"], q["blocks"], q["pv"], n_iter_metropolis=n_iter)
        assert mh.K == 138
        new, acc = mh.sample(q["snc"], {k: v.copy() for k, v in q["dl"].items()}, iteration=3)
        out.append((new, acc))
    (n0, a0), (n1, a1) = out
    assert a0 == a1
    nacc = sum(int(np.sum(v)) for v in a0.values())
    assert 0 < nacc < 138 * n_iter, nacc              # both branches of the decision exercised
    for sp in ("EE", "BB"):
        np.testing.assert_array_equal(n0[sp], n1[sp])
