"""GPU: the matrix-core Legendre stage (gs_sht_set_mfma: plan-time lambda / F1 /
F2 tables, v_mfma_f64_16x16x4_f64 contractions per m with the batch's maps as
columns).

* Small sizes: against the oracle (dense direct sums, oracle/sht.py) at 1e-11,
  every ncomp, both layouts, iter 0 / 3, odd and even l_max (partial blocks,
  partial 16-pair tiles).
* N_side 256 / l_max 512 (the HEAD masked configuration): against the on-the-
  fly recurrence kernels at 1e-12 relative (the same recurrence values, another
  summation order), spin 0 / 2 / TEB, beam and weights.
* A map of a batch is bit-identical to the same map transformed alone (any
  batch size, including maps past a 16-column group).
* The masked context: chains of a batch on the table path equal one-chain
  contexts forced onto it (sht_mode="mfma"), bit for bit.
"""
import numpy as np
import pytest

from oracle import harmonic as H
from oracle import sht as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _rand_alm(L, ncomp, rng):
    ls, ms = O._cidx(L)
    a = rng.standard_normal((ncomp, len(ls))) + 1j * rng.standard_normal((ncomp, len(ls)))
    a[:, ms == 0] = a[:, ms == 0].real
    return a


def _oracle_maps(a3, N, L, ncomp):
    if ncomp == 1:
        return O.alm2map(a3[0], N, L)[None]
    if ncomp == 2:
        full = np.concatenate([np.zeros((1, a3.shape[1]), dtype=complex), a3], axis=0)
        return O.alm2map(full, N, L)[1:]
    return O.alm2map(a3, N, L)


def _oracle_alm(maps, N, L, ncomp, it):
    if ncomp == 1:
        return O.map2alm(maps[0], N, L, iter=it)[None]
    if ncomp == 2:
        full = np.concatenate([np.zeros((1, maps.shape[1])), maps], axis=0)
        return O.map2alm(full, N, L, iter=it)[1:]
    return O.map2alm(maps, N, L, iter=it)


CASES = [(4, 8), (4, 11), (8, 16), (8, 23), (16, 32), (16, 37)]


@pytest.mark.parametrize("N,L", CASES)
@pytest.mark.parametrize("ncomp", [1, 2, 3])
def test_mfma_alm2map_vs_oracle(N, L, ncomp):
    from gibbssampler_amd.sht import HealpixSHT
    sht = HealpixSHT(N, L).set_mfma(True)
    assert sht.mfma[0] and sht.mfma[1] > 0
    rng = np.random.default_rng(100 * N + L + ncomp)
    a = _rand_alm(L, ncomp, rng)
    want = _oracle_maps(a, N, L, ncomp)
    got_c = sht.alm2map(torch.from_numpy(a).cuda(), ncomp=ncomp, layout="complex").cpu().numpy().reshape(ncomp, -1)
    ar = np.stack([H.complex_to_real(x, L) for x in a])
    got_r = sht.alm2map(torch.from_numpy(ar).cuda(), ncomp=ncomp, layout="real").cpu().numpy().reshape(ncomp, -1)
    scale = np.abs(want).max()
    np.testing.assert_allclose(got_c, want, rtol=0, atol=1e-11 * scale)
    np.testing.assert_allclose(got_r, want, rtol=0, atol=1e-11 * scale)


@pytest.mark.parametrize("N,L", CASES)
@pytest.mark.parametrize("ncomp", [1, 2, 3])
@pytest.mark.parametrize("it", [0, 3])
def test_mfma_map2alm_vs_oracle(N, L, ncomp, it):
    from gibbssampler_amd.sht import HealpixSHT
    sht = HealpixSHT(N, L).set_mfma(True)
    rng = np.random.default_rng(7 * N + L + ncomp + it)
    maps = rng.standard_normal((ncomp, 12 * N * N))
    want = _oracle_alm(maps, N, L, ncomp, it)
    got = sht.map2alm(torch.from_numpy(maps).cuda(), iter=it, ncomp=ncomp, layout="complex").cpu().numpy()
    got = got.reshape(ncomp, -1)
    scale = np.abs(want).max()
    np.testing.assert_allclose(got, want, rtol=0, atol=1e-11 * scale)
    gr = sht.map2alm(torch.from_numpy(maps).cuda(), iter=it, ncomp=ncomp, layout="real").cpu().numpy()
    wr = np.stack([H.complex_to_real(x, L) for x in want])
    np.testing.assert_allclose(gr.reshape(ncomp, -1), wr, rtol=0, atol=1e-11 * scale * 2)


@pytest.mark.parametrize("ncomp", [1, 2, 3])
def test_mfma_matches_recurrence_nside256(ncomp):
    """the HEAD masked configuration: table path vs the on-the-fly kernels"""
    from gibbssampler_amd.sht import HealpixSHT
    N, L = 256, 512
    a_sht = HealpixSHT(N, L)
    m_sht = HealpixSHT(N, L).set_mfma(True)
    g = torch.Generator(device="cuda").manual_seed(11)
    B = 5
    alm = torch.randn((B, ncomp, (L + 1) ** 2), dtype=torch.float64, device="cuda", generator=g)
    maps = torch.randn((B, ncomp, 12 * N * N), dtype=torch.float64, device="cuda", generator=g)
    w = torch.rand((ncomp, 12 * N * N), dtype=torch.float64, device="cuda", generator=g)
    bl = torch.rand(L + 1, dtype=torch.float64, device="cuda", generator=g)
    for beam in (None, bl):
        want = a_sht.alm2map_batch(alm, ncomp, bl=beam)
        got = m_sht.alm2map_batch(alm, ncomp, bl=beam)
        err = (got - want).abs().max().item() / want.abs().max().item()
        assert err < 1e-12, err
    for wts, it in ((None, 0), (None, 3), (w, 0)):
        want = a_sht.map2alm_batch(maps, ncomp, iter=it, weights=wts)
        got = m_sht.map2alm_batch(maps, ncomp, iter=it, weights=wts)
        err = (got - want).abs().max().item() / want.abs().max().item()
        assert err < 1e-12, (it, wts is not None, err)


@pytest.mark.parametrize("ncomp", [1, 2, 3])
def test_mfma_batch_bit_identical(ncomp):
    """map b of a batch (37 maps: two full 16-column groups of spin 2 / one and a
    part of spin 0, plus a partial one) = that map transformed alone"""
    from gibbssampler_amd.sht import HealpixSHT
    N, L = 16, 37
    sht = HealpixSHT(N, L).set_mfma(True)
    g = torch.Generator(device="cuda").manual_seed(5)
    B = 37
    alm = torch.randn((B, ncomp, (L + 1) ** 2), dtype=torch.float64, device="cuda", generator=g)
    maps = torch.randn((B, ncomp, 12 * N * N), dtype=torch.float64, device="cuda", generator=g)
    mb = sht.alm2map_batch(alm, ncomp)
    ab = sht.map2alm_batch(maps, ncomp, iter=3)
    for b in (0, 15, 16, 36):
        one = sht.alm2map_batch(alm[b:b + 1], ncomp)
        assert torch.equal(mb[b], one[0]), f"alm2map map {b}"
        one = sht.map2alm_batch(maps[b:b + 1], ncomp, iter=3)
        assert torch.equal(ab[b], one[0]), f"map2alm map {b}"


@pytest.mark.parametrize("mfma", [True, False])
@pytest.mark.parametrize("ncomp,N,L,B,zero", [(2, 16, 37, 5, "cap"), (1, 16, 37, 3, "cap"), (3, 8, 20, 2, "cap"),
                                              (2, 64, 128, 4, "cap"), (2, 64, 128, 3, "band"), (1, 64, 128, 2, "band"),
                                              (2, 32, 64, 2, "none"), (2, 32, 64, 2, "all")])
def test_apply_weighted_equals_two_transforms(mfma, ncomp, N, L, B, zero):
    """the fused operator pass (maps on chip) = alm2map(beamed) then the weighted
    map2alm = the analysis of the pre-weighted maps, bit for bit, on the table
    path and on the recurrence path.  Zero weights on the polar caps / an
    equatorial band (whole ring pairs and 16-pair tiles without weight, which
    the table path skips) / nowhere / everywhere."""
    from gibbssampler_amd.data import pixel_cos_theta
    from gibbssampler_amd.sht import HealpixSHT
    sht = HealpixSHT(N, L).set_mfma(mfma)
    g = torch.Generator(device="cuda").manual_seed(11)
    npix = 12 * N * N
    alm = torch.randn((B, ncomp, (L + 1) ** 2), dtype=torch.float64, device="cuda", generator=g)
    w = torch.rand((ncomp, npix), dtype=torch.float64, device="cuda", generator=g)
    if zero == "cap":
        w[:, : npix // 7] = 0.0
    elif zero == "band":
        w[:, torch.from_numpy(np.abs(pixel_cos_theta(N)) <= 0.2).cuda()] = 0.0
    elif zero == "all":
        w.zero_()
    bl = torch.linspace(1.0, 0.3, L + 1, dtype=torch.float64, device="cuda")
    maps = sht.alm2map_batch(alm, ncomp, bl=bl)
    want = sht.map2alm_batch(maps, ncomp, weights=w)
    pre = sht.map2alm_batch(maps * w, ncomp)          # no weights: nothing skipped
    assert torch.equal(want, pre)
    got = sht.apply_weighted_batch(alm, ncomp, w, bl=bl)
    assert torch.equal(got, want)
    for b in (0, B - 1):
        assert torch.equal(sht.apply_weighted_batch(alm[b:b + 1], ncomp, w, bl=bl)[0], got[b]), b


@pytest.mark.parametrize("ncomp,beam", [(1, False), (2, True), (3, True), (2, False)])
def test_mfma_real_input_equals_complex_input(ncomp, beam):
    """the table synthesis reading the real layout (and beam) itself = the same
    coefficients given in the complex layout (the separate input pass), bit for
    bit: m = 0 (b a_l0, 0), m > 0 ((b a_re) / sqrt 2, (b a_im) / sqrt 2)"""
    from gibbssampler_amd.sht import HealpixSHT
    N, L, B = 16, 37, 5
    sht = HealpixSHT(N, L).set_mfma(True)
    g = torch.Generator(device="cuda").manual_seed(21)
    a = torch.randn((B, ncomp, (L + 1) ** 2), dtype=torch.float64, device="cuda", generator=g)
    bl = torch.linspace(1.0, 0.2, L + 1, dtype=torch.float64, device="cuda") if beam else None
    ls, ms = np.meshgrid(np.arange(L + 1), np.arange(L + 1), indexing="ij")
    keep = ls >= ms
    ls, ms = ls[keep], ms[keep]
    ci = ms * (2 * L + 1 - ms) // 2 + ls                  # complex (healpy) index
    order = np.argsort(ci)
    ls, ms, ci = ls[order], ms[order], ci[order]
    r = np.where(ms == 0, ls, 2 * ci - (L + 1))
    re = a[..., torch.from_numpy(r).cuda()]
    im = a[..., torch.from_numpy(np.where(ms == 0, 0, r + 1)).cuda()]
    b = bl[torch.from_numpy(ls).cuda()] if beam else torch.ones(len(ls), dtype=torch.float64, device="cuda")
    m0 = torch.from_numpy(ms == 0).cuda()
    IS2 = 0.70710678118654752440
    cre = torch.where(m0, b * re, (b * re) * IS2)
    cim = torch.where(m0, torch.zeros_like(im), (b * im) * IS2)
    ac = torch.complex(cre, cim).contiguous()
    want = sht.alm2map_batch(ac, ncomp, layout="complex")
    got = sht.alm2map_batch(a, ncomp, bl=bl)
    assert torch.equal(got, want)


def test_mfma_round_trip_and_adjoint_nside256():
    """band-limited round trip (iter 3) and exact adjointness on the table path"""
    from gibbssampler_amd.sht import HealpixSHT
    N, L = 256, 512
    sht = HealpixSHT(N, L).set_mfma(True)
    npix = 12 * N * N
    g = torch.Generator(device="cuda").manual_seed(3)
    a = torch.randn((2, 2, (L + 1) ** 2), dtype=torch.float64, device="cuda", generator=g)
    m = torch.randn((2, 2, npix), dtype=torch.float64, device="cuda", generator=g)
    Am = sht.alm2map_batch(a, 2)
    At = sht.map2alm_batch(m, 2) * (npix / (4 * np.pi))
    lhs = float((Am * m).sum())
    rhs = float((a * At).sum())
    assert abs(lhs - rhs) / (abs(lhs) + abs(rhs)) < 1e-12
    ls = np.concatenate([np.arange(L + 1)] + [np.repeat(np.arange(mm, L + 1), 2) for mm in range(1, L + 1)])
    # spin 2: l < 2 has no spin-2 harmonic (not recoverable), so the band starts at l = 2
    band = torch.from_numpy(((ls >= 2) & (ls <= int(1.5 * N))).astype(np.float64)).cuda()
    ab = a * band
    back = sht.map2alm_batch(sht.alm2map_batch(ab, 2), 2, iter=3)
    err = (back - ab).abs().max().item() / ab.abs().max().item()
    # HEALPix quadrature is approximate: the same bound as the recurrence path's
    # round trip (tests/test_gpu_sht.py::test_round_trip_fullsize)
    assert err < 1e-4, err


@pytest.mark.parametrize("kind", ["aux", "mala", "pcg"])
def test_masked_batch_on_tables_equals_single(kind):
    """4 chains on the table path (auto for >= 4 chains) = one-chain contexts
    forced onto it, bit for bit (aux CR, MALA accept, the device PCG)"""
    from gibbssampler_amd import _capi
    from gibbssampler_amd.masked import MaskedCR
    N, L = 16, 32
    rng = np.random.default_rng(9)
    npix = 12 * N * N
    th, _ = O.pixel_angles(N)
    mask = (np.abs(np.cos(th)) > 0.2).astype(float)
    maps = rng.standard_normal((3, npix)) * np.array([[30.0], [0.3], [0.3]])
    ell = np.arange(L + 1)
    bl = np.exp(-0.5 * ell * (ell + 1) * (0.05 / np.sqrt(8 * np.log(2))) ** 2)
    dl = np.stack([np.where(ell >= 2, 10.0 * (np.maximum(ell, 1) / 100) ** 0.5, 0), np.where(ell >= 2, 0.01, 0.0)])
    s0 = rng.standard_normal((4, 2, (L + 1) ** 2)) * np.array([[0.05], [0.005]])
    pix = {"Q": maps[1], "U": maps[2]}
    kw = {"aux": dict(gibbs_cr=True, n_gibbs=2), "mala": dict(gibbs_cr=False, ula=True, tau=0.3),
          "pcg": dict(gibbs_cr=False, ula=False, pcg_accuracy=1e-9)}[kind]
    args = dict(mask=mask, nfields=2, rng="native", seed=77, **kw)
    batch = MaskedCR(pix, 40.0 ** 2, 0.2 ** 2, bl, L, N, chain=2, nchains=4, **args)
    assert batch.sht_tables
    dlb = torch.from_numpy(np.stack([dl * (1 + 0.1 * b) for b in range(4)])).cuda()
    sb = torch.from_numpy(np.ascontiguousarray(s0)).cuda()
    if kind == "pcg":
        out = batch.pcg_solve(dlb, batch.pcg_rhs(dlb, iteration=3))
    else:
        code = _capi.GS_MCR_AUX if kind == "aux" else _capi.GS_MCR_MALA
        batch.step(code, dlb, sb, iteration=3)
        out = sb
    for b in (0, 3):
        one = MaskedCR(pix, 40.0 ** 2, 0.2 ** 2, bl, L, N, chain=2 + b, sht_mode="mfma", **args)
        assert one.sht_tables
        d1 = dlb[b].contiguous()
        if kind == "pcg":
            x1 = one.pcg_solve(d1, one.pcg_rhs(d1, iteration=3))
        else:
            x1 = sb.new_tensor(s0[b])
            one.step(code, d1, x1, iteration=3)
        assert torch.equal(out[b], x1), f"chain {b}"
