"""Chains batched through the SHT-bound (masked) path.

The reference runs many independent chains as separate SLURM tasks
(job-script.sh:6-8), each calling healpy's transforms for its own maps.  Here a
context holds B chains and every transform is ONE batched SHT over the B maps.
The contract: chain b of a batch is bit-identical to a one-chain run of global
chain id chain0 + b (the one-chain runs are pinned to the oracle and the
reference's masked goldens in tests/test_gpu_masked.py).  Checked for:
  * the batched transforms themselves (alm2map / map2alm / iter / weights /
    beam, spin 0 / 2 / TEB, small-map segmented and single-walk launch shapes);
  * every masked CR kind (aux, over-relaxation, MALA, aux + MALA), the device
    PCG (per-chain convergence) and RJPO, the pixel-domain MH sweep (f2);
  * the drivers: MaskedRunner (centered) and MaskedMHRunner (ASIS, NC).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import sht as O  # noqa: E402

pytestmark = pytest.mark.gpu

B = 4
CHAIN0 = 3


def _problem(N=8, L=16, seed=3):
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
    s0 = rng.standard_normal((B, 3, (L + 1) ** 2)) * np.array([[3.0], [0.05], [0.005]])
    return N, L, mask, maps, ntemp, npol, bl, dl, s0


# ---- the batched transforms ---------------------------------------------------------
@pytest.mark.parametrize("N,L", [(8, 16), (64, 128), (256, 512)])
@pytest.mark.parametrize("nc", [1, 2, 3])
def test_sht_batch_bit_identical(N, L, nc):
    from gibbssampler_amd.sht import HealpixSHT
    from gibbssampler_amd import _capi
    sht = HealpixSHT(N, L)
    lib = sht.lib
    nb = 3
    npix, NR = 12 * N * N, (L + 1) ** 2
    g = torch.Generator(device="cuda").manual_seed(7)
    alm = torch.randn((nb, nc, NR), dtype=torch.float64, device="cuda", generator=g)
    maps = torch.randn((nb, nc, npix), dtype=torch.float64, device="cuda", generator=g)
    w = torch.rand((nc, npix), dtype=torch.float64, device="cuda", generator=g)
    bl = torch.rand(L + 1, dtype=torch.float64, device="cuda", generator=g)
    sp = _capi.stream_ptr()
    # synthesis (+ beam)
    for beam in (None, bl):
        out = torch.empty((nb, nc, npix), dtype=torch.float64, device="cuda")
        _capi.check(lib.gs_sht_alm2map_batch(sht.handle, nb, nc, _capi.GS_ALM_REAL, _capi.ptr(alm), _capi.ptr(beam),
                                             _capi.ptr(out), sp), "alm2map_batch")
        for b in range(nb):
            one = sht.alm2map_beamed(alm[b], beam, ncomp=nc) if beam is not None else sht.alm2map(alm[b], ncomp=nc)
            assert torch.equal(out[b].reshape(one.shape), one), f"alm2map map {b} beam {beam is not None}"
    # analysis: iter 0 / 3, weighted
    for it in (0, 3):
        out = torch.empty((nb, nc, NR), dtype=torch.float64, device="cuda")
        _capi.check(lib.gs_sht_map2alm_batch(sht.handle, nb, nc, _capi.GS_ALM_REAL, _capi.ptr(maps), None,
                                             _capi.ptr(out), it, sp), "map2alm_batch")
        for b in range(nb):
            one = sht.map2alm(maps[b], iter=it, ncomp=nc)
            assert torch.equal(out[b].reshape(one.shape), one), f"map2alm iter {it} map {b}"
    out = torch.empty((nb, nc, NR), dtype=torch.float64, device="cuda")
    _capi.check(lib.gs_sht_map2alm_batch(sht.handle, nb, nc, _capi.GS_ALM_REAL, _capi.ptr(maps), _capi.ptr(w),
                                         _capi.ptr(out), 0, sp), "map2alm_batch weighted")
    for b in range(nb):
        one = sht.map2alm_weighted(maps[b], w, ncomp=nc)
        assert torch.equal(out[b].reshape(one.shape), one), f"weighted map {b}"


def test_sht_batch_reserve_in_capture_errors():
    """a batch larger than the reserved workspace inside a capture is refused
    (no allocation while capturing); after gs_sht_reserve it captures."""
    from gibbssampler_amd.sht import HealpixSHT
    from gibbssampler_amd import _capi
    N, L = 8, 16
    sht = HealpixSHT(N, L)
    alm = torch.zeros((5, 2, (L + 1) ** 2), dtype=torch.float64, device="cuda")
    maps = torch.empty((5, 2, 12 * N * N), dtype=torch.float64, device="cuda")
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        _capi.check(sht.lib.gs_sht_reserve(sht.handle, 5, _capi.stream_ptr()), "reserve")
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            _capi.check(sht.lib.gs_sht_alm2map_batch(sht.handle, 5, 2, _capi.GS_ALM_REAL, _capi.ptr(alm), None,
                                                     _capi.ptr(maps), _capi.stream_ptr()), "alm2map_batch")
        g.replay()
    torch.cuda.synchronize()
    assert torch.all(maps == 0)


# ---- masked CR kinds -------------------------------------------------------------------
def _crs(kind_kw, F=2, rng="native", sht_mode="recurrence", **kw):
    from gibbssampler_amd.masked import MaskedCR
    N, L, mask, maps, ntemp, npol, bl, dl, s0 = _problem()
    pix = {"T": maps[0], "Q": maps[1], "U": maps[2]}
    # the same Legendre stage for the batch and the one-chain contexts (the
    # table path's summation order differs from the recurrence kernels')
    args = dict(mask=mask, nfields=F, rng=rng, seed=4242, sht_mode=sht_mode, **kind_kw, **kw)
    batch = MaskedCR(pix, ntemp, npol, bl, L, N, chain=CHAIN0, nchains=B, **args)
    ones = [MaskedCR(pix, ntemp, npol, bl, L, N, chain=CHAIN0 + b, **args) for b in range(B)]
    rows = [1, 2] if F == 2 else [0, 1, 2]
    return batch, ones, dl, s0[:, rows], L


def _dlt(cr, dl, nch):
    spec = ("EE", "BB") if cr.F == 2 else ("TT", "EE", "BB", "TE")
    one = np.stack([dl[k] for k in spec])
    # a different D_l per chain (chain b scaled), so the batch's per-chain data paths are exercised
    arr = np.stack([one * (1.0 + 0.1 * b) for b in range(nch)])
    return torch.from_numpy(arr).cuda()


@pytest.mark.parametrize("sht_mode", ["recurrence", "mfma"])
@pytest.mark.parametrize("kind,F", [("aux", 2), ("aux", 3), ("over", 2), ("over", 3), ("mala", 2),
                                    ("aux_mala", 2)])
def test_masked_cr_batch_equals_single(kind, F, sht_mode):
    from gibbssampler_amd import _capi
    kw = {"aux": dict(gibbs_cr=True, n_gibbs=2), "over": dict(gibbs_cr=True, overrelaxation=True, n_gibbs=2),
          "mala": dict(gibbs_cr=False, ula=True, tau=0.3), "aux_mala": dict(gibbs_cr=True, ula=True, tau=0.3)}[kind]
    code = {"aux": _capi.GS_MCR_AUX, "over": _capi.GS_MCR_OVERRELAX, "mala": _capi.GS_MCR_MALA,
            "aux_mala": _capi.GS_MCR_AUX_MALA}[kind]
    batch, ones, dl, s0, L = _crs(kw, F=F, sht_mode=sht_mode)
    assert batch.sht_tables == (sht_mode == "mfma")
    it = 7
    dlb = _dlt(batch, dl, B)
    sb = torch.from_numpy(np.ascontiguousarray(s0)).cuda()
    for _ in range(2):                       # two calls: v carries over (over-relaxation)
        batch.step(code, dlb, sb, iteration=it)
    acc_b = batch._acc.cpu().numpy()
    for b in range(B):
        s1 = sb.new_tensor(s0[b])
        for _ in range(2):
            ones[b].step(code, dlb[b].contiguous(), s1, iteration=it)
        assert torch.equal(sb[b], s1), f"chain {b}"
        assert int(ones[b]._acc.item()) == int(acc_b[b])
    if kind in ("mala", "aux_mala"):
        assert len(set(acc_b.tolist())) >= 1


@pytest.mark.parametrize("sht_mode", ["recurrence", "mfma"])
@pytest.mark.parametrize("F", [2, 3])
def test_pcg_batch_equals_single(F, sht_mode):
    """the batched device CG (per-chain scalars and convergence) = each chain's
    own solve, bit for bit; iteration counts per chain equal."""
    batch, ones, dl, s0, L = _crs(dict(gibbs_cr=False, ula=False), F=F, pcg_accuracy=1e-9, sht_mode=sht_mode)
    it = 2
    dlb = _dlt(batch, dl, B)
    xb = batch.pcg_solve(dlb, batch.pcg_rhs(dlb, iteration=it))
    its_b = batch.pcg_iterations_chains[-1]
    assert batch.pcg_launched[-1] >= max(its_b)
    for b in range(B):
        d1 = dlb[b].contiguous()
        x1 = ones[b].pcg_solve(d1, ones[b].pcg_rhs(d1, iteration=it))
        assert torch.equal(xb[b], x1), f"chain {b}"
        assert ones[b].pcg_iterations[-1] == its_b[b]


def test_rj_batch_equals_single():
    batch, ones, dl, s0, L = _crs(dict(gibbs_cr=False, ula=False, rj=True), F=2, pcg_accuracy=0.0, pcg_maxiter=6)
    it = 3
    dlb = _dlt(batch, dl, B)
    sb = torch.from_numpy(np.ascontiguousarray(s0)).cuda()
    batch.rj_step(dlb, sb, iteration=it)
    acc_b = batch._acc.cpu().numpy()
    lr_b = batch._lr.cpu().numpy()
    for b in range(B):
        s1 = sb.new_tensor(s0[b])
        ones[b].rj_step(dlb[b].contiguous(), s1, iteration=it)
        assert torch.equal(sb[b], s1), f"chain {b}"
        assert int(ones[b]._acc.item()) == int(acc_b[b])
        assert float(ones[b]._lr.item()) == float(lr_b[b])


def _mh_setup(batch_cr, L):
    from gibbssampler_amd.masked import PixelMH
    bins = {"EE": np.arange(L + 2), "BB": np.array([0, 2, 5, 9, 13, L + 1])}
    blocks = {"EE": np.array([2, 6, L + 1]), "BB": np.array([2, 3, 4, 5])}
    ell = np.arange(2, L + 1)
    pv = {"EE": (0.05 * 10.0 * (ell / 100.0) ** 0.5) ** 2, "BB": np.full(len(bins["BB"]) - 3, (0.2 * 0.01) ** 2)}
    return PixelMH(batch_cr, bins, blocks, pv), bins, blocks, pv


def test_pixel_mh_batch_equals_single():
    from gibbssampler_amd.masked import PixelMH
    batch, ones, dl, s0, L = _crs(dict(gibbs_cr=False, ula=False), F=2)
    mhb, bins, blocks, pv = _mh_setup(batch, L)
    it = 5
    start = {"EE": dl["EE"][:L + 1].copy(), "BB": np.array([np.mean(dl["BB"][bins["BB"][i]:bins["BB"][i + 1]])
                                                           for i in range(len(bins["BB"]) - 1)])}
    inits = [{k: v * (1.0 + 0.05 * b) for k, v in start.items()} for b in range(B)]
    cur_b = mhb.plan.dl_tensor(inits)
    s_nc = torch.from_numpy(np.ascontiguousarray(s0 * 30.0)).cuda()
    out_b, fl_b = mhb.sweep_t(s_nc, cur_b, it)
    out_b, fl_b = out_b.cpu().numpy(), fl_b.cpu().numpy().copy()
    for b in range(B):
        mh1 = PixelMH(ones[b], bins, blocks, pv)
        cur1 = mh1.plan.dl_tensor(inits[b])[0]
        o1, f1 = mh1.sweep_t(s_nc[b].contiguous(), cur1, it)
        np.testing.assert_array_equal(out_b[b], o1.cpu().numpy(), err_msg=f"chain {b}")
        np.testing.assert_array_equal(fl_b[b], f1.cpu().numpy(), err_msg=f"chain {b}")


# ---- drivers ---------------------------------------------------------------------------
@pytest.mark.parametrize("sht_mode", ["recurrence", "mfma"])
def test_masked_runner_batch_equals_single(sht_mode):
    """MaskedRunner (the a12 ladder's aux + MALA composition, the C_l draw):
    chains 0 and B - 1 of a B-chain run equal one-chain runs."""
    from gibbssampler_amd.masked import MaskedRunner
    batch, ones, dl, s0, L = _crs(dict(gibbs_cr=True, ula=True, n_gibbs=1), F=2, sht_mode=sht_mode)
    bins = {"EE": np.arange(L + 2), "BB": np.arange(L + 2)}
    init = {"EE": dl["EE"][:L + 1], "BB": dl["BB"][:L + 1]}
    hb, ab, _, _ = MaskedRunner(batch, bins).run(init, 3, s0)
    for b in (0, B - 1):
        h1, a1, _, _ = MaskedRunner(ones[b], bins).run(init, 3, s0[b])
        for sp in h1:
            np.testing.assert_array_equal(hb[sp][:, b], h1[sp], err_msg=f"chain {b} {sp}")
        np.testing.assert_array_equal(ab[:, b], a1)


@pytest.mark.parametrize("sht_mode", ["recurrence", "mfma"])
@pytest.mark.parametrize("kind", ["asis", "noncentered"])
def test_masked_mh_runner_batch_equals_single(kind, sht_mode):
    """MaskedMHRunner: ASIS (over-relaxed aux CR + C_l draw + pixel MH +
    re-centring) and NC (PCG + pixel MH), chains 0 and B - 1 vs one-chain runs."""
    from gibbssampler_amd.masked import MaskedMHRunner, KIND_PCG, cr_kind
    kw = dict(gibbs_cr=True, overrelaxation=True, n_gibbs=2, ula=True) if kind == "asis" else \
        dict(gibbs_cr=False, ula=False)
    batch, ones, dl, s0, L = _crs(kw, F=2, pcg_accuracy=1e-6, sht_mode=sht_mode)
    _, bins, blocks, pv = _mh_setup(batch, L)
    ck = cr_kind(True, True, True) if kind == "asis" else KIND_PCG
    start = {"EE": dl["EE"][:L + 1].copy(), "BB": np.array([np.mean(dl["BB"][bins["BB"][i]:bins["BB"][i + 1]])
                                                           for i in range(len(bins["BB"]) - 1)])}
    rb = MaskedMHRunner(kind, batch, bins, blocks, pv, cr_kind_=ck).run(start, 2, s_init=s0 if kind == "asis" else None)
    for b in (0, B - 1):
        r1 = MaskedMHRunner(kind, ones[b], bins, blocks, pv, cr_kind_=ck).run(
            start, 2, s_init=s0[b] if kind == "asis" else None)
        for sp in r1[0]:
            np.testing.assert_array_equal(rb[0][sp][:, b], r1[0][sp], err_msg=f"chain {b} {sp}")
            np.testing.assert_array_equal(rb[1][sp][:, b], r1[1][sp], err_msg=f"chain {b} {sp} accepts")


def test_surface_masked_nchains():
    """the drop-in class with a mask and nchains > 1 (the NotImplementedError of
    r03 lifted): histories carry the chain axis, chain b = a one-chain sampler
    of chain0 + b."""
    from gibbssampler_amd.gibbs import CenteredGibbs
    N, L, mask, maps, ntemp, npol, bl, dl, s0 = _problem()
    init = {"EE": dl["EE"][:L + 1], "BB": dl["BB"][:L + 1]}
    kw = dict(mask_path=mask, polarization=True, n_iter=2, gibbs_cr=True, ula=False, rng="native", seed=9)
    cg = CenteredGibbs({"Q": maps[1], "U": maps[2]}, ntemp, npol, 4.0, N, L, 12 * N * N, nchains=3, chain0=1,
                       skymap_init=s0[:3, 1:], **kw)
    h, acc, _, _ = cg.run(init)
    assert h["EE"].shape == (3, 3, L + 1)
    one = CenteredGibbs({"Q": maps[1], "U": maps[2]}, ntemp, npol, 4.0, N, L, 12 * N * N, nchains=1, chain0=3,
                        skymap_init=s0[2, 1:], **kw)
    h1, _, _, _ = one.run(init)
    np.testing.assert_array_equal(h["EE"][:, 2], h1["EE"])
    np.testing.assert_array_equal(h["BB"][:, 2], h1["BB"])


def test_surface_default_mode_batch_equals_single_of_resolved_mode():
    """with the default sht_mode ("auto") a 4-chain batch resolves to
    the matrix-core tables and a one-chain run to the recurrence, so the batch
    reproduces a one-chain run of the same chain id only when that run is given
    the batch's resolved mode -- passed through the drop-in class (sht_mode=)."""
    from gibbssampler_amd.gibbs import CenteredGibbs
    N, L, mask, maps, ntemp, npol, bl, dl, s0 = _problem()
    init = {"EE": dl["EE"][:L + 1], "BB": dl["BB"][:L + 1]}
    kw = dict(mask_path=mask, polarization=True, n_iter=2, gibbs_cr=True, ula=True, rng="native", seed=9)
    cg = CenteredGibbs({"Q": maps[1], "U": maps[2]}, ntemp, npol, 4.0, N, L, 12 * N * N, nchains=4, chain0=1,
                       skymap_init=s0[:4, 1:], **kw)
    assert cg.constrained_sampler.sht_tables          # auto at B = 4: tables
    h, acc, _, _ = cg.run(init)
    for mode, tables in (("auto", False), ("mfma", True)):
        one = CenteredGibbs({"Q": maps[1], "U": maps[2]}, ntemp, npol, 4.0, N, L, 12 * N * N, nchains=1, chain0=3,
                            skymap_init=s0[2, 1:], sht_mode=mode, **kw)
        assert one.constrained_sampler.sht_tables == tables
        h1, a1, _, _ = one.run(init)
        if tables:
            np.testing.assert_array_equal(h["EE"][:, 2], h1["EE"])
            np.testing.assert_array_equal(h["BB"][:, 2], h1["BB"])
            np.testing.assert_array_equal(acc[:, 2], a1)
        else:                                          # the other Legendre stage: ~1e-12 apart
            np.testing.assert_allclose(h["EE"][:, 2], h1["EE"], rtol=1e-8)
            np.testing.assert_allclose(h["BB"][:, 2], h1["BB"], rtol=1e-8)


@pytest.mark.parametrize("driver", ["centered", "noncentered", "asis"])
def test_tt_pixel_batch_equals_single(driver):
    """the pixel-domain TT model (f4) batched: chains 0 and B - 1 of a B-chain
    run equal one-chain runs (masked: PCG / aux CR, C_l draw, pixel MH)."""
    from gibbssampler_amd.tt import TTModel
    N, L, mask, maps, ntemp, npol, bl, dl, s0 = _problem()
    bins = np.arange(L + 2)
    pv = (0.05 * 1000.0) ** 2 * np.ones(L - 1)
    kw = dict(mask=mask, rng="native", seed=21, blocks=np.arange(2, L + 2), proposal_variances=pv,
              pcg_accuracy=1e-8, sht_mode="recurrence")
    init = dl["TT"][:L + 1]

    def go(m):
        if driver == "centered":
            return m.run_centered(init, 2)[0]
        if driver == "noncentered":
            return m.run_noncentered(init, 2)[0]
        return m.run_asis(init, 2, gibbs_cr=True)[0]

    hb = go(TTModel(maps[0], ntemp, bl, L, N, bins, chain=4, nchains=B, **kw))
    for b in (0, B - 1):
        h1 = go(TTModel(maps[0], ntemp, bl, L, N, bins, chain=4 + b, **kw))
        np.testing.assert_array_equal(hb[:, b], h1, err_msg=f"chain {b}")
