"""Workgroup timeline of one headline CR sweep (build variant with
-DGS_SWEEP_WGTIME, tools/build_variants.sh): per physical workgroup its start
and end (s_memrealtime, 100 MHz) and CU / XCC; prints the launch span, the
workgroup durations, and the average number of resident sweep workgroups per
CU over the span in 10 slices -- how much of the kernel is its tail.

usage (GPU box): python tools/sweep_timeline.py build_variants/lib_wgtime.so [nchains]"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gibbssampler_amd import _capi  # noqa: E402
from gibbssampler_amd.problem import synthetic_problem  # noqa: E402
from gibbssampler_amd.samplers import BatchedRunner  # noqa: E402


def main(lib, nch="32"):
    nch = int(nch)
    _capi._lib = None
    L = _capi.load(lib)
    P = synthetic_problem(1024, 512, 3, seed=0)
    r = BatchedRunner("noncentered", P["lmax"], P["nside"], 3, nch, P["bl"], P["noise_var"], P["bins"], P["d_alm"],
                      blocks=P["blocks"], proposal_variances=P["proposal_variances"], rng="native", seed=5,
                      store_skymap=False)
    r.init(P["dls_init"])
    for _ in range(30):
        r.step()
    torch.cuda.synchronize()
    n = 16384
    buf = (ctypes.c_ulonglong * (4 * n))()
    fn = L.gs_debug_sweep_timeline
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    fn.restype = ctypes.c_int
    _capi.check(fn(buf, n), "gs_debug_sweep_timeline")
    a = np.frombuffer(buf, dtype=np.uint64).reshape(n, 4).astype(np.int64)
    a = a[a[:, 1] > 0]
    out = os.environ.get("SWEEP_TL_NPY")
    if out:
        np.save(out, a)
    t0 = a[:, 0].min()
    st, en = (a[:, 0] - t0) / 100.0, (a[:, 1] - t0) / 100.0      # microseconds
    hw, xcc = a[:, 2], a[:, 3] & 15
    cu = ((hw >> 8) & 15) | (((hw >> 13) & 7) << 4) | ((hw >> 12) & 1) << 7
    ncu = len(np.unique(xcc * 256 + cu))
    span = en.max()
    dur = en - st
    print(f"{len(a)} workgroups on {ncu} CUs, span {span:.1f} us; duration mean {dur.mean():.1f} "
          f"p10 {np.percentile(dur, 10):.1f} p90 {np.percentile(dur, 90):.1f} max {dur.max():.1f} us")
    edges = np.linspace(0, span, 11)
    for k in range(10):
        a0, a1 = edges[k], edges[k + 1]
        ov = np.clip(np.minimum(en, a1) - np.maximum(st, a0), 0, None).sum() / (a1 - a0)
        print(f"  {a0:7.1f}-{a1:7.1f} us: {ov / ncu:5.2f} workgroups per CU resident")
    # the most workgroups any CU held at once, and how often each count occurs
    key = xcc * 256 + cu
    mx = []
    for k in np.unique(key):
        sel = key == k
        ev = sorted([(t, 1) for t in st[sel]] + [(t, -1) for t in en[sel]], key=lambda e: (e[0], e[1]))
        c = best = 0
        for _, dlt in ev:
            c += dlt
            best = max(best, c)
        mx.append(best)
    mx = np.array(mx)
    print("  max concurrent workgroups per CU:", {int(v): int((mx == v).sum()) for v in np.unique(mx)})
    for x in range(8):
        sel = xcc == x
        print(f"  XCC {x}: {sel.sum():5d} wgs, last end {en[sel].max():7.1f} us, first start {st[sel].min():6.1f}")


if __name__ == "__main__":
    main(*sys.argv[1:])
