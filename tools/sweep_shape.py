"""A/B of the CR-sweep workgroup shape at the bench configuration (one process,
interleaved): GS_SWEEP_TW=1 (1 tile x 4 chunks, partials summed in LDS) vs 4
(4 tiles x 1 chunk).  Each shape: one BatchedRunner, K NC steps captured in a
hipGraph, replays alternated; prints median ms per step and sweep time.

usage (GPU box): python tools/sweep_shape.py [steps] [rounds]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gibbssampler_amd.problem import synthetic_problem  # noqa: E402
from gibbssampler_amd.samplers import BatchedRunner  # noqa: E402


def main(steps=20, rounds=7):
    P = synthetic_problem(1024, 512, 3, seed=0)
    runners = {}
    for tw in ("1", "4"):
        os.environ["GS_SWEEP_TW"] = tw
        r = BatchedRunner("noncentered", P["lmax"], P["nside"], 3, 32, P["bl"], P["noise_var"], P["bins"], P["d_alm"],
                          blocks=P["blocks"], proposal_variances=P["proposal_variances"], rng="native", seed=5)
        r.init(P["dls_init"])
        r.step()
        r.capture_steps(steps, time_sweeps=True, time_every=5)
        runners[tw] = r
    res = {k: [] for k in runners}
    sw = {k: [] for k in runners}
    for rnd in range(rounds):
        for k, r in runners.items():
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            r.plan.sweep_timing("resume")
            e0.record()
            r.step()
            e1.record()
            torch.cuda.synchronize()
            if rnd:
                res[k].append(e0.elapsed_time(e1) / steps)
    for k, r in runners.items():
        ms, n = r.plan.sweep_timing(False)
        print(f"GS_SWEEP_TW={k}: {np.median(res[k]) * 1e3:7.1f} us/step (min {min(res[k]) * 1e3:7.1f}), "
              f"sweep {ms / max(n, 1) * 1e3:7.1f} us avg over {n}")


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
