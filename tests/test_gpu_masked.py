"""GPU: the masked CR samplers (gs_masked_cr through gibbssampler_amd.masked.MaskedCR).

Replay mode against the reference-generated fixtures (same numpy draws, same
algebra: a9 aux-variable, a10 over-relaxation, a11 MALA incl. both accept
branches, a12 composition) and native mode against the oracle's restatement
of the device Philox streams (EB and the TEB generalisation).

VERDICT r04 item 1: every replay / oracle test runs on both Legendre stages --
``sht_mode`` "recurrence" (the on-the-fly VALU kernels, a one-chain context's
"auto") and "mfma" (the matrix-core table path that "auto" picks from 4 chains,
i.e. what every batched masked bench line runs) -- against the same fixtures
and tolerances, and a 4-chain replay batch on tables is checked chain by chain
against the reference's fixtures (chain 0) and the oracle (chains 1-3)."""
import os

import numpy as np
import pytest

from oracle import masked as MK
from oracle import sht as O

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_masked_eb_N8_L16.npz")
TOL = dict(rtol=1e-9)
MODES = ["recurrence", "mfma"]


@pytest.fixture(params=MODES)
def sht_mode(request):
    return request.param


@pytest.fixture(scope="module")
def g():
    return dict(np.load(GOLDEN))


def _cr(g, sht_mode="recurrence", **kw):
    from gibbssampler_amd.masked import MaskedCR
    pix = {"Q": g["Q"], "U": g["U"]}
    cr = MaskedCR(pix, 40.0 ** 2, g["noise_pol"], g["bl"], int(g["L"]), int(g["nside"]), mask=g["mask"],
                  sht_mode=sht_mode, **kw)
    assert cr.sht_tables == (sht_mode == "mfma")
    return cr


def _dls(g):
    return {"EE": g["dl_EE"], "BB": g["dl_BB"]}


def _sold(g):
    return {"EE": g["s_old_E"].copy(), "BB": g["s_old_B"].copy()}


def _close(got, want):
    np.testing.assert_allclose(got, want, rtol=1e-9, atol=1e-11 * np.abs(want).max())


def test_constants(g, sht_mode):
    cr = _cr(g, sht_mode)
    assert cr.mu[1] == pytest.approx(float(g["mu"]), rel=1e-15)
    g2 = cr.second_part_grad().cpu().numpy()
    _close(g2[0], g["second_part_grad_E"])
    _close(g2[1], g["second_part_grad_B"])


def test_a9_replay(g, sht_mode):
    cr = _cr(g, sht_mode, n_gibbs=int(g["a9_ngibbs"]))
    np.random.seed(int(g["a9_seed"]))
    s, acc = cr.sample_gibbs_change_variable(_dls(g), _sold(g))
    assert acc == 1
    _close(s["EE"], g["a9_E"])
    _close(s["BB"], g["a9_B"])


def test_a10_replay(g, sht_mode):
    cr = _cr(g, sht_mode, n_gibbs=int(g["a10_ngibbs"]), overrelaxation=True, alpha=float(g["a10_alpha"]))
    np.random.seed(int(g["a10_seed"]))
    s, acc = cr.overrelaxation_sampler(_dls(g), _sold(g))
    assert acc == 1
    _close(s["EE"], g["a10_E"])
    _close(s["BB"], g["a10_B"])


def test_a11_gradient(g, sht_mode):
    cr = _cr(g, sht_mode, gibbs_cr=False, ula=True)
    gE, gB, pE, pB = cr.compute_gradient_mala(_dls(g), _sold(g))
    _close(gE, g["a11_gradE"])
    _close(gB, g["a11_gradB"])
    _close(pE, g["a11_sEpix"])
    _close(pB, g["a11_sBpix"])


@pytest.mark.parametrize("variant", ["a11", "a11b"])
def test_a11_mala_replay(g, variant, sht_mode):
    tau = float(g["a11_tau"]) if variant == "a11" else float(g["a11b_tau"])
    cr = _cr(g, sht_mode, gibbs_cr=False, ula=True, tau=tau)
    start = _sold(g) if variant == "a11" else {"EE": g["a9_E"], "BB": g["a9_B"]}
    for k, sd in enumerate(g[variant + "_seeds"]):
        np.random.seed(int(sd))
        s, acc = cr.sample_mala(_dls(g), start)
        assert acc == int(g[variant + "_accept"][k])
        _close(s["EE"], g[variant + "_E"][k])
        _close(s["BB"], g[variant + "_B"][k])


def test_a12_composition_replay(g, sht_mode):
    cr = _cr(g, sht_mode, gibbs_cr=True, ula=True, n_gibbs=int(g["a12_ngibbs"]))
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
def test_aux_native_vs_oracle(F, over, sht_mode):
    from gibbssampler_amd.masked import MaskedCR
    N, L, mask, maps, ntemp, npol, bl, dl, s0 = _teb_problem()
    seed, it, chain, ng = 4242, 7, 3, 2
    pix = {"T": maps[0], "Q": maps[1], "U": maps[2]}
    cr = MaskedCR(pix, ntemp, npol, bl, L, N, mask=mask, nfields=F, n_gibbs=ng, overrelaxation=over, rng="native",
                  seed=seed, chain=chain, sht_mode=sht_mode)
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


def test_mala_native_vs_oracle(sht_mode):
    from gibbssampler_amd.masked import MaskedCR
    N, L, mask, maps, ntemp, npol, bl, dl, s0 = _teb_problem(seed=5)
    seed, it, chain = 99, 4, 1
    for tau in (1e-4, 0.6):
        cr = MaskedCR({"Q": maps[1], "U": maps[2]}, ntemp, npol, bl, L, N, mask=mask, nfields=2, gibbs_cr=False,
                      ula=True, tau=tau, rng="native", seed=seed, chain=chain, sht_mode=sht_mode)
        cr.iteration = it
        s, acc = cr.sample_mala(dl, {"EE": s0[1], "BB": s0[2]})
        mm = MK.MaskedModel(L, N, 2, bl, maps, np.stack([mask / ntemp, mask / npol, mask / npol]))
        want, wacc, lr = MK.mala(mm, np.stack([dl["EE"], dl["BB"]]), s0[1:], MK.NativeDraws(seed, chain, it, L, 12 * N * N),
                                 float(npol[0]), tau=tau)
        assert acc == wacc
        np.testing.assert_allclose(cr.last_log_ratio(), lr, rtol=1e-8, atol=1e-8)
        _close(s["EE"], want[0])
        _close(s["BB"], want[1])


def test_masked_centered_driver_replay(g, sht_mode):
    """CenteredGibbs(mask_path=..., gibbs_cr=True) end to end on the device:
    GibbsSampler.run_polarization with the a9 CR and the invgamma C_l draw,
    against the reference driver (start map injected for the qcinv init)."""
    from gibbssampler_amd.gibbs import CenteredGibbs
    L, N = int(g["L"]), int(g["nside"])
    cg = CenteredGibbs({"Q": g["Q"], "U": g["U"]}, np.full(12 * N * N, 40.0 ** 2), g["noise_pol"],
                       float(g["fwhm_deg"]), N, L, 12 * N * N, mask_path=g["mask"], polarization=True,
                       bins={"EE": g["bins_EE"], "BB": g["bins_BB"]}, n_iter=int(g["drv_iters"]), gibbs_cr=True,
                       overrelaxation=False, ula=False, rng="replay", n_gibbs=int(g["drv_ngibbs"]),
                       skymap_init={"EE": g["s_old_E"], "BB": g["s_old_B"]}, sht_mode=sht_mode)
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


def test_f1_pcg_rhs_replay(g, sht_mode):
    """the right-hand side the device builds = the reference's b_fluctuations
    (captured from its qcinv call) + b A^T N^-1 d, same numpy draws."""
    cr = _cr(g, sht_mode, gibbs_cr=False, ula=False)
    np.random.seed(int(g["pcg_seed"]))
    rhs = cr.pcg_rhs(_dl_t(cr, _dls(g))).cpu().numpy()
    g2 = cr.second_part_grad().cpu().numpy()
    _close(rhs[0] - g2[0], g["pcg_bfluct_E"])
    _close(rhs[1] - g2[1], g["pcg_bfluct_B"])


def test_f1_pcg_solve_vs_oracle(g, sht_mode):
    import torch
    cr = _cr(g, sht_mode, gibbs_cr=False, ula=False)
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
def test_f1_pcg_sample_native_vs_oracle(F, sht_mode):
    from gibbssampler_amd.masked import MaskedCR
    N, L, mask, maps, ntemp, npol, bl, dl, s0 = _teb_problem(seed=7)
    seed, it, chain = 31, 2, 5
    cr = MaskedCR({"T": maps[0], "Q": maps[1], "U": maps[2]}, ntemp, npol, bl, L, N, mask=mask, nfields=F,
                  gibbs_cr=False, ula=False, rng="native", seed=seed, chain=chain, pcg_accuracy=1e-13,
                  sht_mode=sht_mode)
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
def test_rj_sample_vs_oracle(F, rng, sht_mode):
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
                  gibbs_cr=False, ula=False, rng=rng, seed=seed, chain=chain, pcg_accuracy=0.0, pcg_maxiter=6, rj=True,
                  sht_mode=sht_mode)
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


def test_f1_pcg_driver_replay_vs_oracle(g, sht_mode):
    """CenteredGibbs(mask, gibbs_cr=False, ula=False): PCG init CR + PCG CR +
    invgamma draws (HEAD's default masked path) against the oracle chain."""
    from gibbssampler_amd.gibbs import CenteredGibbs
    L, N = int(g["L"]), int(g["nside"])
    bins = {"EE": g["bins_EE"], "BB": g["bins_BB"]}
    cg = CenteredGibbs({"Q": g["Q"], "U": g["U"]}, np.full(12 * N * N, 40.0 ** 2), g["noise_pol"],
                       float(g["fwhm_deg"]), N, L, 12 * N * N, mask_path=g["mask"], polarization=True, bins=bins,
                       n_iter=3, gibbs_cr=False, ula=False, rng="replay", sht_mode=sht_mode)
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


def test_f2_pixel_mh_replay(g, sht_mode):
    """the device likelihood and one MH sweep = the reference's
    PolarizationNonCenteredClsSampler.sample(all_sph=False) (fixture f2_*)."""
    from gibbssampler_amd.masked import PixelMH
    bins, blocks, pv = _f2_parts(g)
    mh = PixelMH(_cr(g, sht_mode, gibbs_cr=False, ula=False), bins, blocks, pv)
    snc = {"EE": g["f2_snc_E"], "BB": g["f2_snc_B"]}
    init = {"EE": g["init_EE"].copy(), "BB": g["init_BB"].copy()}
    assert mh.compute_log_likelihood(init, snc) == pytest.approx(float(g["f2_lik0"]), rel=1e-11)
    np.random.seed(int(g["f2_seed"]))
    new, acc = mh.sample(snc, init)
    _close(new["EE"], g["f2_EE"])
    _close(new["BB"], g["f2_BB"])
    assert acc["EE"] == list(g["f2_acc_EE"]) and acc["BB"] == list(g["f2_acc_BB"])


def test_f2_pixel_mh_native_vs_oracle(g, sht_mode):
    from gibbssampler_amd.masked import PixelMH
    bins, blocks, pv = _f2_parts(g)
    seed, chain, it = 77, 3, 5
    cr = _cr(g, sht_mode, gibbs_cr=False, ula=False, rng="native", seed=seed, chain=chain)
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
def test_f2_masked_noncentered_driver_vs_oracle(g, rng, sht_mode):
    """NonCenteredGibbs(mask_path=...): per iteration the PCG CR, C^-1/2, the
    pixel MH sweep (NonCenteredGibbs.py:529-571), against the oracle chain."""
    smp = _masked_mh_sampler(g, "NonCenteredGibbs", 3, rng=rng, seed=19, sht_mode=sht_mode)
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
def test_f2_masked_asis_driver_vs_oracle(g, gibbs_cr, sht_mode):
    """ASIS(mask_path=...): CR (PCG, or the aux + MALA composition with its
    PCG start map), centred C_l draw, non-centring, pixel MH, re-centring with
    the reference's quirk (ASIS.py:134-226), against the oracle chain."""
    n_gibbs = 2
    smp = _masked_mh_sampler(g, "ASIS", 3, gibbs_cr=gibbs_cr, n_gibbs=n_gibbs, sht_mode=sht_mode)
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
def test_f2_device_sweep_groups_vs_oracle(g, gsopt, n_iter, group_bytes, stage, sht_mode):
    """gs_masked_pixel_mh decides every block on the device from one block
    synthesis + one Gram pass; with a small workspace budget the blocks run in
    groups (one block per group at "1") and the residual is carried between
    groups.  Native streams, n_iter_metropolis 1 and 2, against the oracle's
    full-map likelihood per block (oracle/masked.pixel_mh).  stage "0": the
    block synthesis without the LDS-staged inputs (the large-l_max form)."""
    from gibbssampler_amd.masked import PixelMH
    gsopt.setenv("GS_SHT_BLK_STAGE", stage)
    if group_bytes is not None:
        gsopt.setenv("GS_F2_GROUP_BYTES", group_bytes)
    bins, blocks, pv = _f2_parts(g)
    seed, chain, it = 313, 1, 9
    cr = _cr(g, sht_mode, gibbs_cr=False, ula=False, rng="native", seed=seed, chain=chain)
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
def test_f2_large_group_decisions_equal_one_block_groups(f2_large, gsopt, n_iter, sht_mode):
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
            gsopt.delenv("GS_F2_GROUP_BYTES", raising=False)
        else:
            gsopt.setenv("GS_F2_GROUP_BYTES", group_bytes)
        cr = MaskedCR(q["pix"], 40.0 ** 2, np.full(12 * q["N"] ** 2, 0.2 ** 2), q["bl"], q["L"], q["N"],
                      mask=q["mask"], gibbs_cr=False, ula=False, rng="native", seed=515, chain=2, sht_mode=sht_mode)
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


# ---- a 4-chain replay batch on the matrix-core table path ----------
# With sht_mode "auto" every batched masked run (B >= 4) takes the table Legendre
# stage.  Replay draws for a batch are chain-major (each chain's reference-order
# draws in turn), so chain 0 of a batch step seeded like a fixture IS the
# reference's call and must equal the fixture; chains 1-3 continue numpy's stream
# and are checked against the oracle restatement fed the same stream.
NB = 4


def _mm(g):
    return MK.MaskedModel(int(g["L"]), int(g["nside"]), 2, g["bl"], np.stack([np.zeros(768), g["Q"], g["U"]]),
                          np.stack([np.zeros(768), g["inv_noise_pol"], g["inv_noise_pol"]]))


_KINDS = {
    "a9": lambda g: dict(n_gibbs=int(g["a9_ngibbs"])),
    "a10": lambda g: dict(n_gibbs=int(g["a10_ngibbs"]), overrelaxation=True, alpha=float(g["a10_alpha"])),
    "a11": lambda g: dict(gibbs_cr=False, ula=True, tau=float(g["a11_tau"])),
    "a11b": lambda g: dict(gibbs_cr=False, ula=True, tau=float(g["a11b_tau"])),
    "a12": lambda g: dict(gibbs_cr=True, ula=True, n_gibbs=int(g["a12_ngibbs"])),
}


@pytest.mark.parametrize("kind", sorted(_KINDS))
def test_batch4_replay_tables_cr(g, kind):
    """a9 / a10 / a11 (both MALA branches) / a12 through the ladder, 4 chains on
    tables: chain 0 = the reference fixture, chains 1-3 = the oracle; accept
    flags equal (the MALA decisions are thresholds on log ratios that the table
    and recurrence stages give to ~1e-12 -- any flip would show here)."""
    cfg = _KINDS[kind](g)
    cr = _cr(g, "mfma", nchains=NB, **cfg)
    if kind in ("a11", "a11b"):
        seed = int(g[kind + "_seeds"][0])
        start = _sold(g) if kind == "a11" else {"EE": g["a9_E"], "BB": g["a9_B"]}
        want0 = (g[kind + "_E"][0], g[kind + "_B"][0], int(g[kind + "_accept"][0]))
    else:
        seed = int(g[kind + "_seed"])
        start = _sold(g)
        want0 = (g[kind + "_E"], g[kind + "_B"], int(g["a12_accept"]) if kind == "a12" else 1)
    np.random.seed(seed)
    s, acc = cr.sample(_dls(g), [dict(start) for _ in range(NB)])
    assert acc.shape == (NB,)
    _close(s[0]["EE"], want0[0])
    _close(s[0]["BB"], want0[1])
    assert int(acc[0]) == want0[2]
    mm = _mm(g)
    dlu = np.stack([g["dl_EE"], g["dl_BB"]])
    np.random.seed(seed)
    draws = MK.ReplayDraws()
    s_old = np.stack([start["EE"], start["BB"]])
    full = dict(gibbs_cr=True, overrelaxation=False, ula=False, n_gibbs=1, alpha=-0.995, tau=0.02)
    full.update({k: v for k, v in cfg.items() if k in full})
    for b in range(NB):
        want, wacc = MK.sample_dispatch(mm, dlu, s_old, draws, full["gibbs_cr"], full["overrelaxation"], full["ula"],
                                        full["n_gibbs"], float(g["noise_pol"][0]), alpha=full["alpha"],
                                        tau=full["tau"])
        assert int(acc[b]) == int(wacc), f"chain {b}"
        _close(s[b]["EE"], want[0])
        _close(s[b]["BB"], want[1])


def test_batch4_replay_tables_pcg_rhs(g):
    """the PCG right-hand side of 4 chains on tables: chain 0 = the reference's
    captured qcinv input, chains 1-3 = the oracle's fluctuation term."""
    import torch
    cr = _cr(g, "mfma", nchains=NB, gibbs_cr=False, ula=False)
    np.random.seed(int(g["pcg_seed"]))
    dl = torch.from_numpy(np.ascontiguousarray(np.broadcast_to(np.stack([g["dl_EE"], g["dl_BB"]]),
                                                               (NB, 2, len(g["dl_EE"]))))).cuda()
    rhs = cr.pcg_rhs(dl).cpu().numpy()
    g2 = cr.second_part_grad().cpu().numpy()
    _close(rhs[0, 0] - g2[0], g["pcg_bfluct_E"])
    _close(rhs[0, 1] - g2[1], g["pcg_bfluct_B"])
    mm = _mm(g)
    np.random.seed(int(g["pcg_seed"]))
    draws = MK.ReplayDraws()
    for b in range(NB):
        zp = draws.pixel_normals(2, mm.Npix)
        zs = draws.slot_normals(2, (mm.L + 1) ** 2)
        want = MK.pcg_fluctuation(mm, np.stack([g["dl_EE"], g["dl_BB"]]), zp, zs)
        _close(rhs[b] - g2, want)


def test_batch4_replay_tables_pixel_mh(g):
    """one f2 sweep for 4 chains on tables: chain 0 = the reference's
    PolarizationNonCenteredClsSampler.sample (fixture f2_*), chains 1-3 = the
    oracle's full-map likelihood per block with the continued uniforms."""
    from gibbssampler_amd.masked import PixelMH
    from oracle import reference_eb as RE
    bins, blocks, pv = _f2_parts(g)
    cr = _cr(g, "mfma", nchains=NB, gibbs_cr=False, ula=False)
    mh = PixelMH(cr, bins, blocks, pv)
    import torch
    snc = np.stack([g["f2_snc_E"], g["f2_snc_B"]])
    init = {"EE": g["init_EE"].copy(), "BB": g["init_BB"].copy()}
    cur = mh.plan.dl_tensor([init] * NB)
    np.random.seed(int(g["f2_seed"]))
    out, flags = mh.sweep_t(torch.from_numpy(np.ascontiguousarray(np.broadcast_to(snc, (NB,) + snc.shape))).cuda(),
                            cur, 1)
    new = mh.plan.dl_dicts(out)
    acc = mh.split_accept(flags)
    _close(new[0]["EE"], g["f2_EE"])
    _close(new[0]["BB"], g["f2_BB"])
    assert list(acc["EE"][0]) == list(g["f2_acc_EE"]) and list(acc["BB"][0]) == list(g["f2_acc_BB"])
    mm, model = _oracle_model(g)
    np.random.seed(int(g["f2_seed"]))
    for b in range(NB):
        up, ua = RE.draw_mh_uniforms(model)
        want, wacc = MK.pixel_mh(mm, model, init, snc, u_prop=up, u_accept=ua)
        _close(new[b]["EE"], want["EE"])
        _close(new[b]["BB"], want["BB"])
        assert list(acc["EE"][b]) == list(wacc["EE"]) and list(acc["BB"][b]) == list(wacc["BB"]), f"chain {b}"


def _oracle_batch_mh_chains(kind, g, n_iter, seed, cr="pcg", n_gibbs=1):
    """the oracle's masked NC / ASIS chains for a B-chain replay batch: per
    iteration every stage draws chain-major (CR draws of chains 0..B-1, then the
    C_l draws, then the MH uniforms), as MaskedMHRunner's device batch does."""
    from oracle import reference_eb as RE
    mm, model = _oracle_model(g)
    np.random.seed(seed)
    draws = MK.ReplayDraws()
    init = {"EE": g["init_EE"].copy(), "BB": g["init_BB"].copy()}
    binned = [{k: v.copy() for k, v in init.items()} for _ in range(NB)]
    hist = [{sp: [init[sp].copy()] for sp in model.spectra} for _ in range(NB)]
    accs = [{sp: [] for sp in model.spectra} for _ in range(NB)]
    s = [None] * NB
    if kind == "asis" and cr != "pcg":
        s = [MK.pcg_sample(mm, model.unfold(binned[b]), draws, tol=1e-13)[0] for b in range(NB)]
    for _ in range(n_iter):
        dl = [model.unfold(binned[b]) for b in range(NB)]
        if kind == "noncentered":
            s = [MK.pcg_sample(mm, dl[b], draws, tol=1e-13)[0] for b in range(NB)]
            snc = [MK.noncentre(mm, dl[b], s[b]) for b in range(NB)]
            start = binned
        else:
            if cr == "pcg":
                s = [MK.pcg_sample(mm, dl[b], draws, tol=1e-13)[0] for b in range(NB)]
            else:
                s = [MK.sample_dispatch(mm, dl[b], s[b], draws, gibbs_cr=True, overrelaxation_flag=False, ula=True,
                                        n_gibbs=n_gibbs, noise_pol0=float(g["noise_pol"][0]))[0] for b in range(NB)]
            start = [RE.cls_centered(model, s[b]) for b in range(NB)]
            snc = [MK.noncentre(mm, model.unfold(start[b]), s[b]) for b in range(NB)]
        for b in range(NB):
            up, ua = RE.draw_mh_uniforms(model)
            binned[b], a = MK.pixel_mh(mm, model, start[b], snc[b], u_prop=up, u_accept=ua)
            if kind == "asis":
                s[b] = MK.noncentre(mm, model.unfold(binned[b]), s[b], inverse=False)
            for sp in model.spectra:
                hist[b][sp].append(binned[b][sp].copy())
                accs[b][sp].append(a[sp])
    return hist, accs


@pytest.mark.parametrize("cls,gibbs_cr", [("NonCenteredGibbs", False), ("ASIS", False), ("ASIS", True)])
def test_batch4_replay_tables_mh_drivers(g, cls, gibbs_cr):
    """the masked NonCenteredGibbs / ASIS drivers with 4 chains per context in
    replay mode on tables (the PCG or aux + MALA CR, the C_l draw, non-centring,
    the f2 sweep, re-centring), every chain against the oracle's chain."""
    kw = dict(gibbs_cr=gibbs_cr, n_gibbs=2) if cls == "ASIS" else {}
    smp = _masked_mh_sampler(g, cls, 2, nchains=NB, sht_mode="mfma", **kw)
    assert smp.masked_cr.sht_tables
    init = {"EE": g["init_EE"].copy(), "BB": g["init_BB"].copy()}
    np.random.seed(515)
    out = smp.run(init)
    h, acc = out[0], out[1]
    kind = "noncentered" if cls == "NonCenteredGibbs" else "asis"
    want, wacc = _oracle_batch_mh_chains(kind, g, 2, 515, cr="aux_mala" if gibbs_cr else "pcg", n_gibbs=2)
    for b in range(NB):
        for sp in ("EE", "BB"):
            np.testing.assert_allclose(h[sp][:, b], np.array(want[b][sp]), rtol=1e-7, err_msg=f"chain {b} {sp}")
            np.testing.assert_array_equal(acc[sp][:, b], np.array(wacc[b][sp]), err_msg=f"chain {b} {sp}")


def test_batch4_replay_tables_centered_driver(g):
    """the masked CenteredGibbs driver (a9 CR + inverse-Gamma draw) with 4 chains
    on tables in replay mode, every chain against the oracle's chain."""
    from gibbssampler_amd.gibbs import CenteredGibbs
    from oracle import harmonic as H
    from oracle import reference_eb as RE
    L, N = int(g["L"]), int(g["nside"])
    bins = {"EE": g["bins_EE"], "BB": g["bins_BB"]}
    s0 = np.stack([g["s_old_E"], g["s_old_B"]])
    ng = int(g["drv_ngibbs"])
    cg = CenteredGibbs({"Q": g["Q"], "U": g["U"]}, np.full(12 * N * N, 40.0 ** 2), g["noise_pol"],
                       float(g["fwhm_deg"]), N, L, 12 * N * N, mask_path=g["mask"], polarization=True, bins=bins,
                       n_iter=3, gibbs_cr=True, overrelaxation=False, ula=False, rng="replay", n_gibbs=ng,
                       skymap_init=np.broadcast_to(s0, (NB,) + s0.shape).copy(), nchains=NB, sht_mode="mfma")
    assert cg.constrained_sampler.sht_tables
    np.random.seed(int(g["drv_seed"]))
    h, acc, _, _ = cg.run({"EE": g["init_EE"].copy(), "BB": g["init_BB"].copy()})
    assert np.all(acc == 1)
    mm = _mm(g)
    model = H.Model(L, N, 2, g["bl"], [1.0, 1.0], bins, d_alm=np.zeros((2, (L + 1) ** 2)))
    np.random.seed(int(g["drv_seed"]))
    draws = MK.ReplayDraws()
    binned = [{"EE": g["init_EE"].copy(), "BB": g["init_BB"].copy()} for _ in range(NB)]
    s = [s0.copy() for _ in range(NB)]
    want = [{sp: [binned[b][sp]] for sp in ("EE", "BB")} for b in range(NB)]
    for _ in range(3):
        s = [MK.aux_variable(mm, model.unfold(binned[b]), s[b], ng, draws)[0] for b in range(NB)]
        binned = [RE.cls_centered(model, s[b]) for b in range(NB)]
        for b in range(NB):
            for sp in ("EE", "BB"):
                want[b][sp].append(binned[b][sp])
    for b in range(NB):
        for sp in ("EE", "BB"):
            _close(h[sp][:, b], np.array(want[b][sp]))


@pytest.mark.parametrize("blocks_mfma", ["0", "1"])
def test_f2_large_vs_oracle_tables(f2_large, gsopt, blocks_mfma):
    """the 138-block large-R sweep on the table path: the matrix-core block
    synthesis (GS_SHT_BLOCKS_MFMA 1, single-l blocks: every quad straddles
    block edges) and the recurrence block synthesis (0) against the oracle's
    full-map likelihood per block."""
    from gibbssampler_amd.masked import MaskedCR, PixelMH
    from oracle import harmonic as H
    gsopt.setenv("GS_SHT_BLOCKS_MFMA", blocks_mfma)
    q = f2_large
    N, L = q["N"], q["L"]
    npol = np.full(12 * N * N, 0.2 ** 2)
    cr = MaskedCR(q["pix"], 40.0 ** 2, npol, q["bl"], L, N, mask=q["mask"], gibbs_cr=False, ula=False, rng="native",
                  seed=515, chain=2, sht_mode="mfma")
    mh = PixelMH(cr, q["bins"], q["blocks"], q["pv"])
    new, acc = mh.sample(q["snc"], {k: v.copy() for k, v in q["dl"].items()}, iteration=3)
    zero = np.zeros(12 * N * N)
    mm = MK.MaskedModel(L, N, 2, q["bl"], np.stack([zero, q["pix"]["Q"], q["pix"]["U"]]),
                        np.stack([zero, q["mask"] / npol, q["mask"] / npol]))
    model = H.Model(L, N, 2, q["bl"], [1.0, 1.0], q["bins"], blocks=q["blocks"], proposal_variances=q["pv"],
                    d_alm=np.zeros((2, (L + 1) ** 2)))
    want, wacc = MK.pixel_mh(mm, model, {k: v.copy() for k, v in q["dl"].items()}, q["snc"], seed=515, chain=2,
                             iteration=3)
    assert acc == wacc
    _close(new["EE"], want["EE"])
    _close(new["BB"], want["BB"])


@pytest.mark.parametrize("F", [2, 3])
@pytest.mark.parametrize("over", [False, True])
@pytest.mark.parametrize("N,L", [(8, 16), (64, 128)])
def test_aux_store_per_class_bit_identical(gsopt, F, over, N, L):
    """large single maps (per-class ring stage, the on-the-fly Legendre kernels:
    configs[4]'s path, forced here at small N with GS_SHT_MERGE_RINGS=0): the v | s
    step applied as the synthesis ring stage stores its pixels gives the bits of
    the synthesis, k_mc_v and the analysis in turn (GS_SHT_FUSED_AUX=0)."""
    import torch
    from gibbssampler_amd import _capi
    from gibbssampler_amd.masked import MaskedCR
    _, _, _, _, _, _, _, dl, _ = _teb_problem(N, L)
    rng = np.random.default_rng(N + F)
    npix = 12 * N * N
    th, _ = O.pixel_angles(N)
    mask = (np.abs(np.cos(th)) > 0.2).astype(float)
    maps = rng.standard_normal((3, npix)) * np.array([[30.0], [0.3], [0.3]])
    ntemp = np.full(npix, 40.0 ** 2) * np.linspace(0.9, 1.1, npix)
    npol = np.full(npix, 0.2 ** 2) * np.linspace(1.2, 0.8, npix)
    ell = np.arange(L + 1)
    bl = np.exp(-0.5 * ell * (ell + 1) * (0.07 / np.sqrt(8 * np.log(2))) ** 2)
    s0 = rng.standard_normal((3, (L + 1) ** 2)) * np.array([[3.0], [0.05], [0.005]])
    pix = {"T": maps[0], "Q": maps[1], "U": maps[2]}
    rows = (1, 2) if F == 2 else (0, 1, 2)
    spec = ("EE", "BB") if F == 2 else ("TT", "EE", "BB", "TE")
    gsopt.setenv("GS_SHT_MERGE_RINGS", "0")
    out = []
    for fused in ("1", "0"):
        gsopt.setenv("GS_SHT_FUSED_AUX", fused)
        cr = MaskedCR(pix, ntemp, npol, bl, L, N, mask=mask, nfields=F, n_gibbs=3, overrelaxation=over, rng="native",
                      seed=8, chain=2, sht_mode="recurrence")
        s = torch.from_numpy(np.ascontiguousarray(np.stack([s0[r] for r in rows])[None])).cuda()
        d = torch.from_numpy(np.ascontiguousarray(np.stack([dl[k] for k in spec])[None])).cuda()
        cr.step(_capi.GS_MCR_OVERRELAX if over else _capi.GS_MCR_AUX, d, s, iteration=5)
        out.append((s.cpu().numpy(), cr.v.cpu().numpy()))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    np.testing.assert_array_equal(out[0][1], out[1][1])


@pytest.mark.parametrize("F", [2, 3])
@pytest.mark.parametrize("over", [False, True])
def test_aux_fused_pass_bit_identical(gsopt, F, over):
    """the table path's fused v | s + s | v-analysis pass (gs_sht_aux_pass_batch:
    synthesis, the k_mc_v update in the ring workgroup, analysis) and the reuse of
    the over-relaxation's repeated s | v analysis give the bits of the unfused
    transforms (GS_SHT_FUSED_AUX=0), 4 chains, native streams."""
    import torch
    from gibbssampler_amd import _capi
    from gibbssampler_amd.masked import MaskedCR
    N, L, mask, maps, ntemp, npol, bl, dl, s0 = _teb_problem()
    pix = {"T": maps[0], "Q": maps[1], "U": maps[2]}
    rows = (1, 2) if F == 2 else (0, 1, 2)
    spec = ("EE", "BB") if F == 2 else ("TT", "EE", "BB", "TE")
    out = []
    for fused in ("1", "0"):
        gsopt.setenv("GS_SHT_FUSED_AUX", fused)
        cr = MaskedCR(pix, ntemp, npol, bl, L, N, mask=mask, nfields=F, n_gibbs=3, overrelaxation=over, rng="native",
                      seed=8, chain=2, nchains=4, sht_mode="mfma")
        s = torch.from_numpy(np.ascontiguousarray(np.stack([np.stack([s0[r] for r in rows]) * (1 + 0.1 * b)
                                                            for b in range(4)]))).cuda()
        d = torch.from_numpy(np.ascontiguousarray(np.broadcast_to(np.stack([dl[k] for k in spec]),
                                                                  (4, len(spec), L + 1)))).cuda()
        cr.step(_capi.GS_MCR_OVERRELAX if over else _capi.GS_MCR_AUX, d, s, iteration=5)
        out.append((s.cpu().numpy(), cr.v.cpu().numpy()))
    np.testing.assert_array_equal(out[0][0], out[1][0])
    np.testing.assert_array_equal(out[0][1], out[1][1])
