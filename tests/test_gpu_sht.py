"""GPU: parity of the device SHT (gs_sht_*) with the oracle and analytic answers.

Small sizes: bitwise-independent algorithms (device: scaled recurrence, ring
FFT / Bluestein with aliasing; oracle: dense direct sums) agree to 1e-11
relative.  Full sizes (N_side 256/512, l_max 2 N_side): exact adjointness,
band-limited round trips, and single modes at high (l, m) against
scipy.special.sph_harm_y (which exercises the scaled recurrence near the
poles)."""
import math

import numpy as np
import pytest
import scipy.special as sps

from oracle import harmonic as H
from oracle import sht as O

pytestmark = pytest.mark.gpu


def _torch():
    import torch
    assert torch.cuda.is_available()
    return torch


def _rand_alm(L, ncomp, rng, lmin=0):
    ls, ms = O._cidx(L)
    a = rng.standard_normal((ncomp, len(ls))) + 1j * rng.standard_normal((ncomp, len(ls)))
    a[:, ms == 0] = a[:, ms == 0].real
    a[:, ls < lmin] = 0.0
    return a


def _oracle_maps(a3, N, L, ncomp):
    """oracle maps for ncomp 1 (T), 2 (E,B -> Q,U), 3."""
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


CASES = [(1, 2), (2, 4), (2, 5), (4, 8), (4, 11), (8, 16), (8, 23), (16, 32), (16, 40)]


@pytest.mark.parametrize("N,L", CASES)
@pytest.mark.parametrize("ncomp", [1, 2, 3])
def test_alm2map_vs_oracle(N, L, ncomp):
    torch = _torch()
    from gibbssampler_amd.sht import HealpixSHT
    sht = HealpixSHT(N, L)
    rng = np.random.default_rng(100 * N + L + ncomp)
    a = _rand_alm(L, ncomp, rng)
    want = _oracle_maps(a, N, L, ncomp)
    # complex layout
    got_c = sht.alm2map(torch.from_numpy(a).cuda(), ncomp=ncomp, layout="complex").cpu().numpy().reshape(ncomp, -1)
    # real layout
    ar = np.stack([H.complex_to_real(x, L) for x in a])
    got_r = sht.alm2map(torch.from_numpy(ar).cuda(), ncomp=ncomp, layout="real").cpu().numpy().reshape(ncomp, -1)
    scale = np.abs(want).max()
    np.testing.assert_allclose(got_c, want, rtol=0, atol=1e-11 * scale)
    np.testing.assert_allclose(got_r, want, rtol=0, atol=1e-11 * scale)


@pytest.mark.parametrize("N,L", CASES)
@pytest.mark.parametrize("ncomp", [1, 2, 3])
@pytest.mark.parametrize("it", [0, 3])
def test_map2alm_vs_oracle(N, L, ncomp, it):
    torch = _torch()
    from gibbssampler_amd.sht import HealpixSHT
    sht = HealpixSHT(N, L)
    rng = np.random.default_rng(7 * N + L + ncomp + it)
    maps = rng.standard_normal((ncomp, O.npix(N)))
    want = _oracle_alm(maps, N, L, ncomp, it)
    got = sht.map2alm(torch.from_numpy(maps).cuda(), iter=it, layout="complex", ncomp=ncomp).cpu().numpy()
    got = got.reshape(ncomp, -1)
    scale = np.abs(want).max()
    np.testing.assert_allclose(got, want, rtol=0, atol=1e-11 * scale)
    got_r = sht.map2alm(torch.from_numpy(maps).cuda(), iter=it, layout="real", ncomp=ncomp).cpu().numpy()
    want_r = np.stack([H.complex_to_real(x, L) for x in want])
    np.testing.assert_allclose(got_r.reshape(ncomp, -1), want_r, rtol=0, atol=2e-11 * scale)


def _real_dot(a, b):
    return float((a * b).sum())


@pytest.mark.parametrize("N,L", [(256, 512), (512, 1024), (1024, 2048)])
@pytest.mark.parametrize("ncomp", [1, 3])
def test_adjointness_fullsize(N, L, ncomp):
    """<A a, m> = <a, A^T m> in the real layout, A^T = map2alm(iter=0)/w (exact)."""
    torch = _torch()
    from gibbssampler_amd.sht import HealpixSHT
    sht = HealpixSHT(N, L)
    g = torch.Generator(device="cuda").manual_seed(11)
    a = torch.randn((ncomp, (L + 1) ** 2), generator=g, device="cuda", dtype=torch.float64)
    m = torch.randn((ncomp, 12 * N * N), generator=g, device="cuda", dtype=torch.float64)
    Am = sht.alm2map(a, ncomp=ncomp)
    At = sht.map2alm(m, ncomp=ncomp) * (12 * N * N / (4 * math.pi))
    lhs = float((Am.reshape(-1) * m.reshape(-1)).sum())
    rhs = float((a.reshape(-1) * At.reshape(-1)).sum())
    assert abs(lhs - rhs) <= 1e-10 * (abs(Am).sum().item() ** 0.5 * abs(m).sum().item() ** 0.5)


@pytest.mark.parametrize("N", [64, 256])
def test_round_trip_fullsize(N):
    """band-limited a (l <= 1.5 N): map2alm(alm2map(a), iter=3) ~ a."""
    torch = _torch()
    from gibbssampler_amd.sht import HealpixSHT
    L = 3 * N // 2
    sht = HealpixSHT(N, L)
    rng = np.random.default_rng(N)
    a = _rand_alm(L, 3, rng, lmin=2)
    at = torch.from_numpy(a).cuda()
    mp = sht.alm2map(at, ncomp=3, layout="complex")
    e = []
    for it in (0, 3):
        b = sht.map2alm(mp, iter=it, layout="complex", ncomp=3)
        e.append((b - at).abs().max().item())
    assert e[1] < e[0]
    assert e[1] < 1e-4 * np.abs(a).max()


def _lambda_mp(l, m, x):
    """lambda_lm(x) in 60-digit mpmath arithmetic (no exponent range limit):
    closed-form lambda_mm, then the three-term recurrence in l."""
    import mpmath as mp
    with mp.workdps(60):
        x = mp.mpf(float(x))
        s = mp.sqrt(1 - x * x)
        lmm = (-1) ** m * mp.sqrt((2 * m + 1) / (4 * mp.pi) * mp.factorial(2 * m)) / (2 ** m * mp.factorial(m)) * s ** m
        if l == m:
            return float(lmm)
        p0, p1 = lmm, x * mp.sqrt(2 * m + 3) * lmm
        for k in range(m + 2, l + 1):
            a = mp.sqrt(mp.mpf(4 * k * k - 1) / (k * k - m * m))
            b = mp.sqrt(mp.mpf((k - 1) ** 2 - m * m) / (4 * (k - 1) ** 2 - 1))
            p0, p1 = p1, a * (x * p1 - b * p0)
        return float(p1)


@pytest.mark.parametrize("N,L,modes", [
    (256, 512, [(512, 0), (512, 500), (400, 390), (300, 150), (511, 511)]),
    (512, 1024, [(1024, 1000), (1000, 990), (900, 30), (1024, 1024)]),
    # per-class ring stage with M = 8192 Bluestein rings: the two-level twiddle
    # and phase tables, the Bluestein products inside the FFT passes
    (1024, 2048, [(2048, 0), (2000, 1990), (1500, 700), (700, 3)]),
])
def test_single_modes_vs_scipy(N, L, modes):
    """a single a_lm (l, m) -> 2 Re(a Y_lm) at every pixel of sampled rings,
    including polar rings where lambda_lm ~ sin^m underflows fp64."""
    torch = _torch()
    from gibbssampler_amd.sht import HealpixSHT
    sht = HealpixSHT(N, L)
    z, nphi, phi0, start = O.ring_info(N)
    rings = sorted(set([0, 1, 2, 5, 17, N // 2, N - 1, N, 2 * N - 1, 3 * N, 4 * N - 2]))
    for (l, m) in modes:
        a = np.zeros((1, (L + 1) * (L + 2) // 2), dtype=np.complex128)
        coef = 0.6 + (0.8j if m > 0 else 0.0)
        a[0, m * (2 * L + 1 - m) // 2 + l] = coef
        mp = sht.alm2map(torch.from_numpy(a).cuda(), ncomp=1, layout="complex").cpu().numpy()
        for r in rings:
            th = math.acos(z[r])
            ph = phi0[r] + 2 * np.pi * np.arange(nphi[r]) / nphi[r]
            Y = sps.sph_harm_y(l, m, np.full_like(ph, th), ph)
            if not np.all(np.isfinite(Y)):
                # scipy overflows for m ~ 1000: arbitrary-precision lambda_lm instead
                Y = _lambda_mp(l, m, z[r]) * np.exp(1j * m * ph)
            want = (coef * Y).real * (1.0 if m == 0 else 2.0)
            got = mp[start[r]:start[r] + nphi[r]]
            np.testing.assert_allclose(got, want, rtol=0, atol=1e-10 * max(1.0, np.abs(want).max()))


@pytest.mark.parametrize("thr", [32, 64])
@pytest.mark.parametrize("ncomp", [1, 3])
def test_large_ring_fft_paths_vs_oracle(thr, ncomp, gsopt):
    """The ring-FFT paths N_side >= 2048 takes (rings whose Bluestein length
    exceeds the LDS: split into two half-length Bluesteins in LDS, or the
    global-scratch FFT), exercised at N_side 16 by lowering the LDS threshold
    of the plan (GS_SHT_LDS_FFT_MAX)."""
    torch = _torch()
    from gibbssampler_amd.sht import HealpixSHT
    gsopt.setenv("GS_SHT_LDS_FFT_MAX", str(thr))
    N, L = 16, 40
    sht = HealpixSHT(N, L)
    rng = np.random.default_rng(thr + ncomp)
    a = _rand_alm(L, ncomp, rng)
    want = _oracle_maps(a, N, L, ncomp)
    got = sht.alm2map(torch.from_numpy(a).cuda(), ncomp=ncomp, layout="complex").cpu().numpy().reshape(ncomp, -1)
    np.testing.assert_allclose(got, want, rtol=0, atol=1e-11 * np.abs(want).max())
    maps = rng.standard_normal((ncomp, O.npix(N)))
    want_a = _oracle_alm(maps, N, L, ncomp, 0)
    got_a = sht.map2alm(torch.from_numpy(maps).cuda(), iter=0, layout="complex", ncomp=ncomp).cpu().numpy()
    np.testing.assert_allclose(got_a.reshape(ncomp, -1), want_a, rtol=0, atol=1e-11 * np.abs(want_a).max())


def test_adjointness_nside2048():
    """exact adjointness at N_side 2048 (split-half Bluestein rings in play)."""
    test_adjointness_fullsize(2048, 4096, 1)


SHAPES = [("2,1", "4,1"), ("2,0", "2,1"), ("1,1", "2,0"), ("1,0", "1,1"), ("2,1", "1,0"), ("4,1", "4,0")]


@pytest.mark.parametrize("syn,ana", SHAPES)
@pytest.mark.parametrize("N,L", [(16, 32), (64, 100)])
def test_legendre_launch_shapes_vs_oracle(gsopt, syn, ana, N, L):
    """Every Legendre launch shape the plan may pick (ring groups per lane
    1/2/4 for synthesis and analysis; m paired or not) -- chosen by map size
    for occupancy, forced here with GS_SHT_SYN / GS_SHT_ANA -- against the
    dense oracle (TEB, both directions; 64/100 with several ring groups)."""
    torch = _torch()
    from gibbssampler_amd.sht import HealpixSHT
    gsopt.setenv("GS_SHT_SYN", syn)
    gsopt.setenv("GS_SHT_ANA", ana)
    sht = HealpixSHT(N, L)
    rng = np.random.default_rng(N + L)
    a = _rand_alm(L, 3, rng)
    want = _oracle_maps(a, N, L, 3)
    got = sht.alm2map(torch.from_numpy(a).cuda(), ncomp=3, layout="complex").cpu().numpy().reshape(3, -1)
    np.testing.assert_allclose(got, want, rtol=0, atol=1e-11 * np.abs(want).max())
    maps = rng.standard_normal((3, O.npix(N)))
    wa = _oracle_alm(maps, N, L, 3, 0)
    ga = sht.map2alm(torch.from_numpy(maps).cuda(), iter=0, layout="complex", ncomp=3).cpu().numpy().reshape(3, -1)
    np.testing.assert_allclose(ga, wa, rtol=0, atol=1e-11 * np.abs(wa).max())


@pytest.mark.parametrize("seg", [4, 8, 20])
@pytest.mark.parametrize("ana", ["1,0", "2,1", "4,1"])
@pytest.mark.parametrize("N,L", [(16, 32), (64, 100)])
def test_segmented_analysis_vs_oracle(gsopt, seg, ana, N, L):
    """l-segmented analysis and synthesis (GS_SHT_SEG: every m's l range split
    into segments entered with the plan-time recurrence state; the default for
    small maps) against the dense oracle, for every analysis launch shape, with
    segment starts before, inside and after the polar onsets."""
    torch = _torch()
    from gibbssampler_amd.sht import HealpixSHT
    gsopt.setenv("GS_SHT_SEG", str(seg))
    gsopt.setenv("GS_SHT_ANA", ana)
    gsopt.setenv("GS_SHT_SYN", "1,0")        # the segmented synthesis's shape
    sht = HealpixSHT(N, L)
    rng = np.random.default_rng(seg + N + L)
    for ncomp in (1, 2, 3):
        a = _rand_alm(L, ncomp, rng)
        want = _oracle_maps(a, N, L, ncomp)
        got = sht.alm2map(torch.from_numpy(a).cuda(), ncomp=ncomp, layout="complex").cpu().numpy()
        np.testing.assert_allclose(got.reshape(ncomp, -1), want, rtol=0, atol=1e-11 * np.abs(want).max())
        maps = rng.standard_normal((ncomp, O.npix(N)))
        wa = _oracle_alm(maps, N, L, ncomp, 0)
        ga = sht.map2alm(torch.from_numpy(maps).cuda(), iter=0, layout="complex",
                         ncomp=ncomp).cpu().numpy().reshape(ncomp, -1)
        np.testing.assert_allclose(ga, wa, rtol=0, atol=1e-11 * np.abs(wa).max())


@pytest.mark.parametrize("N,L", [(16, 40), (64, 100)])
def test_ring_two_level_twiddles_vs_oracle(gsopt, N, L):
    """The per-class ring FFTs with the two-level LDS twiddle tables (the
    M = 8192 classes of N_side >= 2048 take them: the full table does not fit
    beside the buffer), forced at small sizes with GS_SHT_RING_TW2 on the
    per-class stage: TEB both directions against the dense oracle."""
    torch = _torch()
    from gibbssampler_amd.sht import HealpixSHT
    gsopt.setenv("GS_SHT_RING_TW2", "1")
    gsopt.setenv("GS_SHT_MERGE_RINGS", "0")
    sht = HealpixSHT(N, L)
    rng = np.random.default_rng(N * L + 2)
    a = _rand_alm(L, 3, rng)
    want = _oracle_maps(a, N, L, 3)
    got = sht.alm2map(torch.from_numpy(a).cuda(), ncomp=3, layout="complex").cpu().numpy().reshape(3, -1)
    np.testing.assert_allclose(got, want, rtol=0, atol=1e-11 * np.abs(want).max())
    maps = rng.standard_normal((3, O.npix(N)))
    wa = _oracle_alm(maps, N, L, 3, 0)
    ga = sht.map2alm(torch.from_numpy(maps).cuda(), iter=0, layout="complex", ncomp=3).cpu().numpy().reshape(3, -1)
    np.testing.assert_allclose(ga, wa, rtol=0, atol=1e-11 * np.abs(wa).max())


@pytest.mark.parametrize("seg", [0, 200])
def test_analysis_launch_shapes_agree_long_l(gsopt, seg):
    """The large-map analysis shapes (4 ring groups per lane, m paired or not;
    unsegmented, or segments over 64 l on the unsegmented kernel) against the
    2-group shape at l_max 512 -- several hundred l per m, onsets spread over
    the range -- for T, EB and TEB: only the partial-sum grouping differs."""
    torch = _torch()
    from gibbssampler_amd.sht import HealpixSHT
    N, L = 128, 512
    rng = np.random.default_rng(512 + seg)
    for ncomp in (1, 2, 3):
        maps = torch.from_numpy(rng.standard_normal((ncomp, 12 * N * N))).cuda()
        res = {}
        for ana in ("4,1", "4,0", "2,1"):
            gsopt.setenv("GS_SHT_SEG", str(seg))
            gsopt.setenv("GS_SHT_ANA", ana)
            sht = HealpixSHT(N, L)
            res[ana] = sht.map2alm(maps, iter=0, layout="complex", ncomp=ncomp).cpu().numpy()
            del sht
        ref = res["2,1"]
        for ana in ("4,1", "4,0"):
            np.testing.assert_allclose(res[ana], ref, rtol=0, atol=1e-12 * np.abs(ref).max())


@pytest.mark.parametrize("N,L,seg", [(256, 512, 64), (256, 512, 16), (512, 1024, 64)])
def test_segmented_analysis_matches_single_walk(gsopt, N, L, seg):
    """At the HEAD masked modes' size (and N_side 512): segmented and
    single-walk analysis and synthesis agree to rounding (the segment states continue the
    same recurrence; only the reduction grouping of a few l differs), iter 0
    and the Jacobi iter 3, TEB."""
    torch = _torch()
    from gibbssampler_amd.sht import HealpixSHT
    rng = np.random.default_rng(N + seg)
    maps = torch.from_numpy(rng.standard_normal((3, 12 * N * N))).cuda()
    alm = torch.from_numpy(_rand_alm(L, 3, rng)).cuda()
    out = {}
    for sg in (0, seg):
        gsopt.setenv("GS_SHT_SEG", str(sg))
        gsopt.setenv("GS_SHT_ANA", "1,0")
        gsopt.setenv("GS_SHT_SYN", "1,0")
        sht = HealpixSHT(N, L)
        out[sg] = [sht.map2alm(maps, iter=it, layout="complex", ncomp=3).cpu().numpy() for it in (0, 3)]
        out[sg].append(sht.alm2map(alm, ncomp=3, layout="complex").cpu().numpy())
        del sht
    for a, b in zip(out[0], out[seg]):
        np.testing.assert_allclose(b, a, rtol=0, atol=1e-12 * np.abs(a).max())


@pytest.mark.parametrize("merge", ["0", "1"])
@pytest.mark.parametrize("N,L", [(16, 40), (64, 128)])
def test_ring_stage_merged_and_per_class_vs_oracle(gsopt, merge, N, L):
    """Small maps run the whole ring stage as one launch (every FFT length in
    one grid, GS_SHT_MERGE_RINGS default on for lengths <= 2048); larger maps
    one launch per length class.  Both against the dense oracle, TEB, both
    directions."""
    torch = _torch()
    from gibbssampler_amd.sht import HealpixSHT
    gsopt.setenv("GS_SHT_MERGE_RINGS", merge)
    sht = HealpixSHT(N, L)
    rng = np.random.default_rng(N + L + int(merge))
    a = _rand_alm(L, 3, rng)
    want = _oracle_maps(a, N, L, 3)
    got = sht.alm2map(torch.from_numpy(a).cuda(), ncomp=3, layout="complex").cpu().numpy().reshape(3, -1)
    np.testing.assert_allclose(got, want, rtol=0, atol=1e-11 * np.abs(want).max())
    maps = rng.standard_normal((3, O.npix(N)))
    wa = _oracle_alm(maps, N, L, 3, 0)
    ga = sht.map2alm(torch.from_numpy(maps).cuda(), iter=0, layout="complex", ncomp=3).cpu().numpy().reshape(3, -1)
    np.testing.assert_allclose(ga, wa, rtol=0, atol=1e-11 * np.abs(wa).max())


@pytest.mark.parametrize("mfma", [False, True])
def test_ring_stage_merged_equals_per_class_n512(gsopt, mfma):
    """N_side 512 (FFT lengths up to M = 4096: the polar Bluestein rings) runs
    the merged ring stage by default since r06; it equals the per-class
    launches (GS_SHT_MERGE_RINGS=0) to rounding -- batched spin-2 maps on both
    Legendre stages, both directions, and the N^-1-weighted operator whose
    constant rings skip the DFTs only in the merged stage."""
    torch = _torch()
    from gibbssampler_amd.sht import HealpixSHT
    from gibbssampler_amd.data import band_mask
    N, L, B = 512, 1024, 3
    g = torch.Generator(device="cuda").manual_seed(5)
    alm = torch.randn((B, 2, (L + 1) ** 2), generator=g, device="cuda", dtype=torch.float64)
    maps = torch.randn((B, 2, 12 * N * N), generator=g, device="cuda", dtype=torch.float64)
    w = torch.from_numpy(np.stack([band_mask(N)] * 2) * 25.0).cuda()
    out = {}
    for mg in ("1", "0"):
        gsopt.setenv("GS_SHT_MERGE_RINGS", mg)
        sht = HealpixSHT(N, L)
        if mfma:
            sht.set_mfma(True)
        out[mg] = [sht.alm2map_batch(alm, 2).cpu().numpy(), sht.map2alm_batch(maps, 2).cpu().numpy(),
                   sht.apply_weighted_batch(alm, 2, w).cpu().numpy()]
        del sht
    for a, b in zip(out["0"], out["1"]):
        np.testing.assert_allclose(b, a, rtol=0, atol=1e-12 * np.abs(a).max())


@pytest.mark.parametrize("N,L,comps", [(256, 512, 2), (512, 1024, 3)])
def test_cpu_baseline_sht_equals_device(N, L, comps):
    """The CPU baseline's transforms (oracle/sht_cpu.cpp: own FFTs and scaled
    recurrence) equal the device SHT at the masked workloads' sizes (1e-10
    relative, both directions): the CPU leg computes the same transform."""
    torch = _torch()
    from gibbssampler_amd.sht import HealpixSHT
    from oracle import sht_cpu as C
    nc = 3 if comps == 3 else 2
    sht = HealpixSHT(N, L)
    rng = np.random.default_rng(N)
    a = np.zeros((3, (L + 1) * (L + 2) // 2), dtype=np.complex128)
    ls, ms = O._cidx(L)
    a[3 - nc:] = rng.normal(size=(nc, len(ls))) + 1j * rng.normal(size=(nc, len(ls)))
    a[:, ms == 0] = a[:, ms == 0].real
    a[1:, ls < 2] = 0
    dev = sht.alm2map(torch.from_numpy(a).cuda(), ncomp=3, layout="complex").cpu().numpy()
    cpu = C.alm2map(a[3 - nc:], N, L, comps=comps)
    np.testing.assert_allclose(cpu, dev[3 - nc:], rtol=0, atol=1e-10 * np.abs(dev).max())
    mp = rng.normal(size=(3, 12 * N * N))
    mp[: 3 - nc] = 0.0
    dev = sht.map2alm(torch.from_numpy(mp).cuda(), iter=0, layout="complex", ncomp=3).cpu().numpy()
    cpu = C.map2alm(mp[3 - nc:], N, L, comps=comps)
    np.testing.assert_allclose(cpu, dev[3 - nc:], rtol=0, atol=1e-10 * np.abs(dev).max())


@pytest.mark.parametrize("N,L", [(64, 100), (256, 512)])
def test_default_small_map_shapes_match_single_walk(gsopt, N, L):
    """The small-map default plan mixes launch shapes over one 32-l segment
    table: synthesis and TEB analysis in 64-l segments with one ring group per
    lane (two table rows per segment), T and spin-2 analysis in 32-l segments
    with two ring groups per lane.  Every ncomp against the unsegmented single
    walk of the same plan shape family, to rounding."""
    torch = _torch()
    from gibbssampler_amd.sht import HealpixSHT
    rng = np.random.default_rng(N + L + 7)
    out = {}
    for mode in ("default", "walk"):
        if mode == "walk":
            gsopt.setenv("GS_SHT_SEG", "0")
            gsopt.setenv("GS_SHT_ANA", "1,0")
            gsopt.setenv("GS_SHT_SYN", "1,0")
        sht = HealpixSHT(N, L)
        res = []
        for ncomp in (1, 2, 3):
            r2 = np.random.default_rng(ncomp)
            maps = torch.from_numpy(r2.standard_normal((ncomp, 12 * N * N))).cuda()
            alm = torch.from_numpy(_rand_alm(L, ncomp, r2)).cuda()
            res.append(sht.map2alm(maps, iter=0, layout="complex", ncomp=ncomp).cpu().numpy())
            res.append(sht.alm2map(alm, ncomp=ncomp, layout="complex").cpu().numpy())
        out[mode] = res
        del sht
    for a, b in zip(out["walk"], out["default"]):
        np.testing.assert_allclose(b, a, rtol=0, atol=1e-12 * np.abs(a).max())


@pytest.mark.parametrize("N,L,ncomp,env", [(16, 32, 2, None), (64, 100, 3, None), (256, 512, 2, None),
                                           (64, 128, 2, "split"), (32, 64, 1, None)])
def test_fused_beam_and_weight_bit_identical(N, L, ncomp, env, gsopt):
    """gs_sht_alm2map_beamed / gs_sht_map2alm_weighted (the masked CR's b s
    synthesis and N^-1-weighted analysis, CenteredGibbs.py:298-299,510-513,698-699)
    equal the separate multiply + plain transform bit for bit: merged and
    per-class ring launches, and ("split") the half-length Bluestein / global
    scratch ring paths forced by a small LDS FFT cap."""
    torch = _torch()
    if env == "split":
        gsopt.setenv("GS_SHT_LDS_FFT_MAX", "64")
        gsopt.setenv("GS_SHT_MERGE_RINGS", "0")
    from gibbssampler_amd.sht import HealpixSHT
    sht = HealpixSHT(N, L)
    rng = np.random.default_rng(7 * N + L + ncomp)
    a = _rand_alm(L, ncomp, rng)
    ar = torch.from_numpy(np.stack([H.complex_to_real(x, L) for x in a])).cuda()
    bl = torch.from_numpy(np.exp(-0.5 * np.arange(L + 1) * (np.arange(L + 1) + 1) * 1e-4) * 1.3).cuda()
    ell = torch.from_numpy(H.slot_ell(L)).cuda()
    want = sht.alm2map(bl[ell][None] * ar, ncomp=ncomp)
    got = sht.alm2map_beamed(ar, bl, ncomp=ncomp)
    torch.cuda.synchronize()
    assert torch.equal(got, want)
    maps = torch.from_numpy(rng.standard_normal((ncomp, 12 * N * N))).cuda()
    w = torch.from_numpy(rng.uniform(0.0, 3.0, (ncomp, 12 * N * N)) * (rng.uniform(size=(ncomp, 12 * N * N)) > 0.2)).cuda()
    want = sht.map2alm(w * maps, iter=0, ncomp=ncomp)
    got = sht.map2alm_weighted(maps, w, ncomp=ncomp)
    torch.cuda.synchronize()
    assert torch.equal(got, want)
