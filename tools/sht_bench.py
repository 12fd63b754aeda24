"""Time the device SHT (alm2map / map2alm) at the BASELINE sizes and check the
large-N_side FFT path (M > 8192, global scratch) for correctness.

usage: python tools/sht_bench.py [--nside 512] [--lmax 1024] [--reps 10] [--big]
Prints one line per (direction, ncomp): ms per transform and achieved fp64
TFLOP/s by SURVEY.md section 8(d)'s count (N_ringpair * N_lm * c, c = 4 spin 0,
16 spin 2 (Q,U), 20 for T,Q,U)."""
import argparse
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gibbssampler_amd.sht import HealpixSHT  # noqa: E402


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def bench(N, L, reps):
    t0 = time.time()
    sht = HealpixSHT(N, L)
    torch.cuda.synchronize()
    print(f"plan N_side={N} l_max={L}: {time.time() - t0:.2f} s, {sht.device_bytes / 2**30:.2f} GiB device tables",
          flush=True)
    nlm = (L + 1) * (L + 2) // 2
    npair = 2 * N
    g = torch.Generator(device="cuda").manual_seed(1)
    for ncomp, c in ((1, 4), (2, 16), (3, 20)):
        a = torch.randn((ncomp, (L + 1) ** 2), generator=g, device="cuda", dtype=torch.float64)
        m = torch.randn((ncomp, 12 * N * N), generator=g, device="cuda", dtype=torch.float64)
        out_m = torch.empty_like(m)
        out_a = torch.empty_like(a)
        ts = timeit(lambda: sht.alm2map(a, ncomp=ncomp, out=out_m), reps)
        ta = timeit(lambda: sht.map2alm(m, ncomp=ncomp, out=out_a), reps)
        fl = npair * nlm * c
        print(f"ncomp={ncomp}: alm2map {ts:8.3f} ms ({fl / ts / 1e9:6.2f} TF/s)   "
              f"map2alm(iter=0) {ta:8.3f} ms ({fl / ta / 1e9:6.2f} TF/s)", flush=True)
    return sht


def bench_batch(N, L, reps, batches, ncomps=(2,), mfma=False, apply=False, band=0.2):
    """batched transforms (gs_sht_*_batch, one launch per stage for B maps): ms per
    batch, ms per map and TF/s; the beam / N^-1 fused forms of the masked CR."""
    from gibbssampler_amd import _capi
    sht = HealpixSHT(N, L)
    if mfma:
        t0 = time.time()
        sht.set_mfma(True)
        torch.cuda.synchronize()
        print(f"Legendre tables: {sht.mfma[1] / 2**30:.2f} GiB, built in {time.time() - t0:.2f} s", flush=True)
    lib = sht.lib
    nlm = (L + 1) * (L + 2) // 2
    npair = 2 * N
    g = torch.Generator(device="cuda").manual_seed(1)
    for ncomp in ncomps:
        c = {1: 4, 2: 16, 3: 20}[ncomp]
        w = torch.rand((ncomp, 12 * N * N), generator=g, device="cuda", dtype=torch.float64)
        bl = torch.rand(L + 1, generator=g, device="cuda", dtype=torch.float64)
        for B in batches:
            a = torch.randn((B, ncomp, (L + 1) ** 2), generator=g, device="cuda", dtype=torch.float64)
            m = torch.randn((B, ncomp, 12 * N * N), generator=g, device="cuda", dtype=torch.float64)
            out_m, out_a = torch.empty_like(m), torch.empty_like(a)
            sp = _capi.stream_ptr()
            syn = lambda: lib.gs_sht_alm2map_batch(sht.handle, B, ncomp, 0, _capi.ptr(a), _capi.ptr(bl),
                                                   _capi.ptr(out_m), sp)
            ana = lambda: lib.gs_sht_map2alm_batch(sht.handle, B, ncomp, 0, _capi.ptr(m), _capi.ptr(w),
                                                   _capi.ptr(out_a), 0, sp)
            ts, ta = timeit(syn, reps), timeit(ana, reps)
            fl = npair * nlm * c * B
            print(f"batch N_side={N} ncomp={ncomp} B={B:3d}: alm2map {ts:8.3f} ms ({ts / B:7.4f} ms/map, "
                  f"{fl / ts / 1e9:6.2f} TF/s)   map2alm {ta:8.3f} ms ({ta / B:7.4f} ms/map, {fl / ta / 1e9:6.2f} TF/s)",
                  flush=True)
            if apply:
                # the masked PCG operator: map2alm(N^-1 alm2map(b a)) with the bench's
                # 80% band mask in N^-1 (gs_sht_apply_weighted_batch)
                from gibbssampler_amd.data import band_mask
                wm = w * torch.from_numpy(band_mask(N, band)).cuda()
                op = lambda: lib.gs_sht_apply_weighted_batch(sht.handle, B, ncomp, _capi.ptr(a), _capi.ptr(bl),
                                                             _capi.ptr(wm), _capi.ptr(out_m), _capi.ptr(out_a), sp)
                to = timeit(op, reps)
                print(f"batch N_side={N} ncomp={ncomp} B={B:3d}: weighted operator (|cos| > {band}) {to:8.3f} ms "
                      f"({to / B:7.4f} ms/map)", flush=True)


def check_big(N, L):
    """adjointness + one single mode at a size whose cap rings need M > 8192."""
    sht = HealpixSHT(N, L)
    g = torch.Generator(device="cuda").manual_seed(3)
    a = torch.randn((3, (L + 1) ** 2), generator=g, device="cuda", dtype=torch.float64)
    m = torch.randn((3, 12 * N * N), generator=g, device="cuda", dtype=torch.float64)
    Am = sht.alm2map(a, ncomp=3)
    At = sht.map2alm(m, ncomp=3) * (12 * N * N / (4 * math.pi))
    lhs = float((Am.reshape(-1) * m.reshape(-1)).sum())
    rhs = float((a.reshape(-1) * At.reshape(-1)).sum())
    rel = abs(lhs - rhs) / (abs(lhs) + abs(rhs))
    print(f"big N_side={N}: adjoint rel diff {rel:.3e}", flush=True)
    assert rel < 1e-11, rel
    # l = 3000, m = 7 single mode on a cap ring with nphi = 4 * 1500 (Bluestein M = 16384)
    from oracle import sht as O
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_gpu_sht import _lambda_mp
    l, mm = 3000, 7
    ac = torch.zeros((1, (L + 1) * (L + 2) // 2), dtype=torch.complex128, device="cuda")
    ac[0, mm * (2 * L + 1 - mm) // 2 + l] = 0.6 + 0.8j
    mp_ = sht.alm2map(ac, ncomp=1, layout="complex").cpu().numpy()
    z, nphi, phi0, start = O.ring_info(N)
    worst = 0.0
    for r in (1499, 1800, 2047, 2048, 4000):
        ph = phi0[r] + 2 * np.pi * np.arange(nphi[r]) / nphi[r]
        want = 2.0 * ((0.6 + 0.8j) * _lambda_mp(l, mm, z[r]) * np.exp(1j * mm * ph)).real
        got = mp_[start[r]:start[r] + nphi[r]]
        worst = max(worst, np.abs(got - want).max())
    print(f"big N_side={N}: single mode l={l} m={mm} max abs err {worst:.3e}", flush=True)
    assert worst < 1e-9


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--nside", type=int, default=512)
    ap.add_argument("--lmax", type=int, default=None)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--big", action="store_true")
    ap.add_argument("--batch", default=None, help="comma-separated batch sizes: batched-transform timings only")
    ap.add_argument("--ncomp", default="2")
    ap.add_argument("--mfma", action="store_true", help="batched timings on the matrix-core table path")
    ap.add_argument("--apply", action="store_true", help="also the fused weighted operator (masked PCG)")
    ap.add_argument("--band", type=float, default=0.2, help="--apply: zero weight where |cos theta| <= band")
    ap.add_argument("--opt", action="append", default=[], help="NAME=VALUE library option (gs_option_set) "
                                                               "before the plan is made, e.g. GS_SHT_ANA=2,1")
    args = ap.parse_args()
    if args.opt:
        from gibbssampler_amd import _capi
        for o in args.opt:
            k, v = o.split("=", 1)
            _capi.set_option(k, v)
    if args.batch:
        bench_batch(args.nside, args.lmax or 2 * args.nside, args.reps, [int(b) for b in args.batch.split(",")],
                    tuple(int(c) for c in args.ncomp.split(",")), mfma=args.mfma, apply=args.apply, band=args.band)
        raise SystemExit(0)
    bench(args.nside, args.lmax or 2 * args.nside, args.reps)
    if args.big:
        check_big(2048, 4096)
