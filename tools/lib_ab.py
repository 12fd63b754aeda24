"""Whole-step A/B of library BUILDS in ONE process (box-to-box spread is up to
~10 % on the headline workload, so builds are compared interleaved): each
library gets its own BatchedRunner (plans bind the library they were created
with) with K steps captured in one hipGraph; the replays alternate over rounds.

usage (GPU box): python tools/lib_ab.py KIND L NSIDE NCHAINS STEPS lib1.so lib2.so ...
  e.g. python tools/lib_ab.py noncentered 1024 512 32 200 gibbssampler_amd/libgibbs_hip.so build_variants/lib_x.so
Prints the median (and min) microseconds per step of each build, and whether
the builds' D_l trajectories are bit-identical to the first one's."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gibbssampler_amd import _capi  # noqa: E402
from gibbssampler_amd.problem import synthetic_problem  # noqa: E402
from gibbssampler_amd.samplers import BatchedRunner  # noqa: E402


def main(kind, L, nside, nch, steps, *libs, rounds=9):
    L, nside, nch, steps = int(L), int(nside), int(nch), int(steps)
    P = synthetic_problem(L, nside, 3, seed=0)
    runners, traces = {}, {}
    for lib in libs:
        _capi._lib = None
        _capi.load(lib, allow_missing=True)
        r = BatchedRunner(kind, P["lmax"], P["nside"], 3, nch, P["bl"], P["noise_var"], P["bins"], P["d_alm"],
                          blocks=P["blocks"], proposal_variances=P["proposal_variances"], rng="native", seed=5,
                          store_skymap=False)
        r.init(P["dls_init"])
        tr = r.plan.zeros(steps, nch, r.plan.nspec, r.plan.maxbins)
        r.capture_steps(steps, trace=tr, trace_capacity=steps)
        runners[lib], traces[lib] = r, tr
    res = {k: [] for k in runners}
    first = {}
    for rnd in range(rounds):
        for k, r in runners.items():
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            r.step()
            e1.record()
            torch.cuda.synchronize()
            if rnd == 0:
                first[k] = traces[k].cpu().numpy().copy()
            else:
                res[k].append(e0.elapsed_time(e1) / steps)
    ref = first[libs[0]]
    for k in runners:
        same = np.array_equal(first[k], ref)
        print(f"{os.path.basename(k):32s} {np.median(res[k]) * 1e3:8.2f} us/step (min {min(res[k]) * 1e3:8.2f})"
              f"  trajectory {'==' if same else '!='} {os.path.basename(libs[0])}", flush=True)


if __name__ == "__main__":
    main(*sys.argv[1:])
