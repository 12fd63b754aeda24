"""GPU: every BASELINE.json config at its own size.

configs[1] and configs[2] are checked natively against the oracle in
tests/test_gpu_scale.py; this file covers the other three:

* configs[0] -- CenteredGibbs temperature-only, N_side 64, l_max 128, 1 chain:
  the TT pixel path (gibbssampler_amd.tt through the class surface: full-sky
  closed-form CR from the T map with adjoint_synthesis_hp iter 3 every
  iteration, CenteredGibbs.py:108-132, and the TT C_l draw, :24-48) for three
  iterations against oracle.masked.tt_chain on the same Philox streams; plus
  the NonCentered TT driver (pixel-likelihood MH, NonCenteredGibbs.py:488-527).
* configs[3] -- ASIS TEB, N_side 512, l_max 1024, a 32-chain plan (one GPU's
  share of 256 chains over 8 GPUs): one gs_step_asis iteration (ASIS.py:134-226:
  centered CR, centered inverse-Wishart / inverse-Gamma draw, non-centring of
  the statistics, NC MH, re-centring with the reference's quirk at
  ASIS.py:203), chains 0 and 31 against the oracle: the centered map, the
  centered D_l, the NC D_l and all accept flags, the re-centred map and its
  statistics.
* configs[4] -- masked CenteredGibbs TEB, N_side 2048, l_max 4096 (f_sky 0.8),
  one aux-variable CR step (CenteredGibbs.py:676-729, n_gibbs 1): the dense
  oracle SHT cannot run at this size, so the step is checked through
  size-independent properties -- exact adjointness of its spin-0 + spin-2 SHT
  pair, the v | s draw recovered to the oracle's Philox normals (and N(0, 1)
  over all 150 M pixels), and the s | v draw against the oracle's per-l block
  algebra on sampled slots given the step's own analysis of v + N^-1 d.

Tolerances: 1e-10 relative for native mode vs the oracle (libm ulps),
SHT-based maps 1e-8 (the TT chain's iter-3 analyses)."""
import math

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import harmonic as H  # noqa: E402
from oracle import masked as MK  # noqa: E402
from oracle import sht as O  # noqa: E402
from tests._util import stats_rows  # noqa: E402

pytestmark = pytest.mark.gpu
SEED = 20261016


# ---- configs[0]: TT, N_side 64, l_max 128 ---------------------------------------------
def _tt_problem():
    from gibbssampler_amd.problem import gauss_beam
    N, L = 64, 128
    npix = 12 * N * N
    rng = np.random.default_rng(64128)
    noise = 40.0 ** 2                                         # config.py:36
    theta, phi = O.pixel_angles(N)
    tmap = 60.0 * np.cos(theta) ** 2 + 25.0 * np.sin(3 * phi) * np.sin(theta) + rng.normal(0, 40.0, npix)
    bins = np.arange(0, L + 2)
    blocks = np.array([2, 40, 80, L + 1])
    dl0 = np.r_[0.0, 0.0, np.full(L - 1, 1000.0)]
    pv = (0.05 * dl0[2:]) ** 2                                # bins >= 2 (config.py:119-132)
    return dict(N=N, L=L, npix=npix, noise=noise, T=tmap, bins=bins, blocks=blocks, init=dl0, pv=pv,
                bl=gauss_beam(math.radians(0.5), L), fwhm=0.5)


@pytest.mark.parametrize("kind", ["centered", "noncentered"])
def test_configs0_tt_fullsize_matches_oracle(kind):
    from gibbssampler_amd.gibbs import CenteredGibbs, NonCenteredGibbs
    q = _tt_problem()
    N, L, npix = q["N"], q["L"], q["npix"]
    noise = np.full(npix, q["noise"])
    n_iter = 3
    if kind == "centered":
        smp = CenteredGibbs(q["T"], noise, noise, q["fwhm"], N, L, npix, polarization=False, bins=q["bins"],
                            n_iter=n_iter, rng="native", seed=SEED)
    else:
        smp = NonCenteredGibbs(q["T"], noise, noise, q["fwhm"], N, L, npix, q["pv"], metropolis_blocks=q["blocks"],
                               polarization=False, bins=q["bins"], n_iter=n_iter, rng="native", seed=SEED)
    assert smp.tt_pixel
    out = smp.run(q["init"].copy())
    mm = MK.tt_model(L, N, q["bl"], q["T"], np.full(npix, 1.0 / q["noise"]))
    model = H.Model(L, N, 1, q["bl"], [1.0], {"TT": q["bins"]}, blocks={"TT": q["blocks"]},
                    proposal_variances={"TT": q["pv"]}, d_alm=np.zeros((1, (L + 1) ** 2)))
    want, wacc, _ = MK.tt_chain(kind, mm, mm, model, {"TT": q["init"]}, n_iter,
                                lambda it: MK.NativeDraws(SEED, 0, it, L, npix), native=(SEED, 0))
    np.testing.assert_allclose(out[0], want, rtol=1e-8, atol=1e-11 * np.abs(want).max())
    if kind == "noncentered":
        np.testing.assert_array_equal(out[1], wacc)
        assert 0 < np.sum(wacc) < np.size(wacc)            # both branches of the MH decision


# ---- configs[3]: ASIS TEB, N_side 512, l_max 1024, 32 chains ------------------------------
def test_configs3_asis_fullsize_matches_oracle():
    from gibbssampler_amd.engine import GibbsPlan
    from gibbssampler_amd.problem import synthetic_problem
    P = synthetic_problem(1024, 512, 3, seed=0)
    m = H.Model(P["lmax"], P["nside"], 3, P["bl"], P["noise_var"], P["bins"], P["blocks"],
                P["proposal_variances"], P["d_alm"])
    nch, it = 32, 6
    p = GibbsPlan(m.L, m.nside, 3, nch, m.bl, m.noise_var, m.bins, blocks=m.blocks,
                  proposal_variances=m.proposal_variances)
    assert p.nacc > 400
    d = p.data_tensor(m.d_alm)
    dl = p.dl_tensor(P["dls_init"])
    dl_tmp = torch.zeros_like(dl)
    s = p.zeros(nch, 3, p.NR)
    acc = p.zeros(nch, p.nacc, dtype=torch.int32)
    # centered map alone (the step's first launch, same counters) for the
    # un-re-centred check, then the whole step with the quirk's re-centring
    s_c, _ = p.cr_sweep(d, p.block_params(0, dl), seed=SEED, iteration=it)
    p.step_asis(d, dl, s, seed=SEED, iteration=it, accept=acc, dl_tmp=dl_tmp, recentre=True)
    st_rc = p.sweep_stats(d, s)
    torch.cuda.synchronize()
    out_c, out_nc = p.dl_dicts(dl_tmp), p.dl_dicts(dl)
    accs = p.split_accept(acc)
    un0 = m.unfold(P["dls_init"])
    M, Lc = H.centered_params(m, un0)
    ell = H.slot_ell(m.L)
    for c in (0, nch - 1):
        z = np.stack([H.cr_normals(SEED, c, it, 0, f, m.L) for f in range(3)])
        ref = H.cr_apply(m, M, Lc, m.d_alm, z)
        np.testing.assert_allclose(s_c[c].cpu().numpy(), ref, rtol=1e-10, atol=1e-12 * np.abs(ref).max())
        stats = H.sweep_stats(m, ref, m.d_alm)
        want_c = H.centered_cls_draw(m, stats, seed=SEED, chain=c, iteration=it)
        for sp in m.spectra:
            np.testing.assert_allclose(out_c[c][sp], want_c[sp], rtol=1e-10, err_msg="centered " + sp)
        # ASIS.py:180-190: the statistics of s_nc = A(C_tmp)^+ s, then the NC MH from C_tmp
        un_c = m.unfold(want_c)
        stats_nc = H.transform_stats(stats, H.chol_pinv(H.cov_chol(m, un_c)))
        want_nc, wacc = H.nc_mh(m, want_c, stats_nc, seed=SEED, chain=c, iteration=it)
        for sp in m.spectra:
            np.testing.assert_allclose(out_nc[c][sp], want_nc[sp], rtol=1e-10, err_msg="noncentered " + sp)
            np.testing.assert_array_equal(accs[sp][c], wacc[sp], err_msg=sp)
        # ASIS.py:203 (quirk): s <- A(C_new) s, on the centered map
        A = H.cov_chol(m, m.unfold(want_nc))
        rc = np.einsum("sfg,gs->fs", A[ell], ref)
        got = s[c].cpu().numpy()
        np.testing.assert_allclose(got, rc, rtol=1e-10, atol=1e-12 * np.abs(rc).max())
        rows = stats_rows(3, H.sweep_stats(m, rc, m.d_alm))
        st_c = st_rc[c].cpu().numpy()
        for r in range(rows.shape[0]):
            np.testing.assert_allclose(st_c[r], rows[r], rtol=1e-10, atol=1e-12 * np.abs(rows[r]).max(),
                                       err_msg=f"re-centred statistic row {r}")
        del got, rc, ref, z


# ---- configs[4]: masked TEB aux-variable CR, N_side 2048, l_max 4096 ----------------------
def test_configs4_masked_aux_step_fullsize():
    from gibbssampler_amd import _capi
    from gibbssampler_amd.masked import MaskedCR
    from gibbssampler_amd.problem import gauss_beam
    from gibbssampler_amd.sht import HealpixSHT
    N, L, F = 2048, 4096, 3
    npix, NR = 12 * N * N, (L + 1) ** 2
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(5)
    # 1) exact adjointness of the step's SHT pair (T spin-0 + Q/U spin-2)
    sht = HealpixSHT(N, L)
    a = torch.randn((F, NR), generator=g, device=dev, dtype=torch.float64)
    mp = torch.randn((F, npix), generator=g, device=dev, dtype=torch.float64)
    lhs = float((sht.alm2map(a, ncomp=F) * mp).sum())
    rhs = float((a * sht.map2alm(mp, ncomp=F)).sum()) * (npix / (4 * math.pi))
    assert abs(lhs - rhs) <= 1e-10 * math.sqrt(float(a.abs().sum()) * float(mp.abs().sum()))
    del a, mp
    # the problem: noise-only data maps, f_sky 0.8 mask (|cos theta| > 0.2), config.py noise levels
    z = torch.from_numpy(np.cos(O.pixel_angles(N)[0])).to(dev)
    mask = (z.abs() > 0.2).double()
    del z
    sig2 = torch.tensor([40.0 ** 2, 0.2 ** 2, 0.2 ** 2], device=dev, dtype=torch.float64)
    maps = torch.randn((3, npix), generator=g, device=dev, dtype=torch.float64) * sig2.sqrt()[:, None] * mask
    bl = gauss_beam(math.radians(0.5), L)
    ll = np.arange(L + 1.0)
    dl = np.zeros((4, L + 1))
    dl[0, 2:], dl[1, 2:], dl[2, 2:] = 1000.0, 10.0 * (ll[2:] / 100.0) ** 0.5, 0.01
    dl[3] = 0.5 * np.sqrt(dl[0] * dl[1])
    cr = MaskedCR({"T": maps[0].cpu().numpy(), "Q": maps[1].cpu().numpy(), "U": maps[2].cpu().numpy()},
                  40.0 ** 2, 0.2 ** 2, bl, L, N, mask=mask.cpu().numpy(), nfields=F, gibbs_cr=True, n_gibbs=1,
                  rng="native", seed=SEED, chain=3)
    dl_t = torch.from_numpy(dl).to(dev)
    s0 = torch.randn((F, NR), generator=g, device=dev, dtype=torch.float64) * 1e-2
    s = s0.clone()
    it = 2
    cr.step(_capi.GS_MCR_AUX, dl_t, s, iteration=it)
    v = cr.v
    # 2) v | s: v = gamma A b s + sqrt(gamma) z, gamma = mu - N^-1 (CenteredGibbs.py:693-700)
    b_t = torch.from_numpy(bl).to(dev)
    ell = torch.from_numpy(H.slot_ell(L)).to(dev)
    Abs = sht.alm2map(s0 * b_t[ell][None], ncomp=F)
    inv = mask[None] / sig2[:, None]
    mu = torch.from_numpy(cr.mu).to(dev)
    gam = mu[:, None] - inv
    zhat = (v - gam * Abs) / gam.sqrt()
    del Abs
    n = zhat.numel()
    mean, var = float(zhat.mean()), float(zhat.var())
    assert abs(mean) < 6.0 / math.sqrt(n) and abs(var - 1.0) < 6.0 * math.sqrt(2.0 / n), (mean, var)
    k0, k1 = H.chain_key(SEED, 3)
    rng = np.random.default_rng(1)
    pix = np.concatenate([np.arange(64), rng.integers(0, npix, 4000), [npix - 1]]).astype(np.uint64)
    for row in range(3):
        w = H.philox4x32_10(pix, row, MK.TAG_AUX_V | (0 << 8), it, k0, k1)
        zo = H.box_muller(*w)[0]
        np.testing.assert_allclose(zhat[row, pix.astype(np.int64)].cpu().numpy(), zo, rtol=0, atol=1e-6,
                                   err_msg=f"row {row}")
    del zhat
    # 3) s | v on sampled slots: s = M (map2alm(v + N^-1 d) / mu) + Lc z (per-l TEB block, kappa = mu / w)
    r_real = sht.map2alm(v + inv * maps, ncomp=F).cpu().numpy()
    mm_model = H.Model(L, N, F, bl, [1.0 / float(cr.mu[k]) for k in range(3)],
                       {sp: np.arange(L + 2) for sp in H.SPECTRA[3]})
    M, Lc = H.centered_params(mm_model, dl)
    i_c = np.concatenate([np.arange(L + 1), rng.integers(L + 1, (L + 1) * (L + 2) // 2, 6000)]).astype(np.uint64)
    ls, ms = H.complex_ell_m(L)
    got = s.cpu().numpy()
    w = H.philox4x32_10(i_c[None, :], np.arange(F, dtype=np.uint64)[:, None],
                        H.TAG_CR | (MK.SUB_S << 8), it, k0, k1)
    z0, z1 = H.box_muller(*w)
    ii = i_c.astype(np.int64)
    for part, zz in ((0, z0), (1, z1)):
        sel = ii if part == 0 else ii[ii > L]
        if part == 1:
            zz = zz[:, ii > L]
        slot = np.where(sel <= L, sel, 2 * sel - (L + 1) + part)
        lv = ls[sel]
        d_eff = r_real[:, slot] / cr.mu[:, None]
        want = np.einsum("sfg,gs->fs", M[lv], d_eff) + np.einsum("sfg,gs->fs", Lc[lv], zz)
        np.testing.assert_allclose(got[:, slot], want, rtol=1e-9, atol=1e-12 * np.abs(want).max(),
                                   err_msg=f"s | v part {part}")
    del ms
