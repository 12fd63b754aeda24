"""A/B of plan-creation settings (library options read when a plan is built,
include/gibbs_capi.h gs_option_set, e.g. GS_SWEEP_TW) on one workload, in ONE process, interleaved
(box-to-box and process-to-process spread is +-5%): each setting gets its own
BatchedRunner with K steps captured in a hipGraph; replays alternate.

usage (GPU box):
  python tools/step_ab.py KIND L NSIDE NCHAINS STEPS "VAR=a" "VAR=b" ...
  e.g.  python tools/step_ab.py noncentered 1024 512 32 200 GS_SWEEP_TW=1 GS_SWEEP_TW=2
(GIBBS_HIP_LIB=<path> switches whole builds instead: tools/build_variants.sh)
The r02 sweep-shape A/B (1 tile x 4 chunks vs 4 x 1, GS_SWEEP_TW) ran this way.
GS_AB_NOSTORE=1 in the environment: runners without the sky-map store."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gibbssampler_amd import _capi  # noqa: E402
from gibbssampler_amd.problem import synthetic_problem  # noqa: E402
from gibbssampler_amd.samplers import BatchedRunner  # noqa: E402


def main(kind, L, nside, nch, steps, *settings, rounds=9):
    L, nside, nch, steps = int(L), int(nside), int(nch), int(steps)
    P = synthetic_problem(L, nside, 3, seed=0)
    runners = {}
    for st in settings:
        k, v = st.split("=", 1)
        old = _capi.get_option(k)
        _capi.set_option(k, v)
        r = BatchedRunner(kind, P["lmax"], P["nside"], 3, nch, P["bl"], P["noise_var"], P["bins"], P["d_alm"],
                          blocks=P["blocks"], proposal_variances=P["proposal_variances"], rng="native", seed=5,
                          store_skymap=os.environ.get("GS_AB_NOSTORE") is None)
        r.init(P["dls_init"])
        r.step()
        r.capture_steps(steps)
        runners[st] = r
        _capi.set_option(k, old)
    res = {k: [] for k in runners}
    for rnd in range(rounds):
        for k, r in runners.items():
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            r.step()
            e1.record()
            torch.cuda.synchronize()
            if rnd:
                res[k].append(e0.elapsed_time(e1) / steps)
    for k in runners:
        print(f"{k:30s} {np.median(res[k]) * 1e3:8.2f} us/step (min {min(res[k]) * 1e3:8.2f})")


if __name__ == "__main__":
    main(*sys.argv[1:])
