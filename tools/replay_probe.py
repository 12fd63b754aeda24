"""Per-replay step time of a captured K-step hipGraph (bench.py's timed graph):
is the first replay of a freshly instantiated graph slower than later ones, and
does uploading the executable graph first (hipGraphUpload) remove it?

usage (GPU box): python tools/replay_probe.py [K] [time_every]"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gibbssampler_amd.problem import synthetic_problem  # noqa: E402
from gibbssampler_amd.samplers import BatchedRunner  # noqa: E402


def timed(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


def main(K=50, every=10):
    K, every = int(K), int(every)
    P = synthetic_problem(1024, 512, 3, seed=0)
    hip = ctypes.CDLL("libamdhip64.so")
    for mode in ("plain", "upload"):
        r = BatchedRunner("noncentered", P["lmax"], P["nside"], 3, 32, P["bl"], P["noise_var"], P["bins"], P["d_alm"],
                          blocks=P["blocks"], proposal_variances=P["proposal_variances"], rng="native", seed=5)
        r.init(P["dls_init"])
        r.capture_steps(5)
        r.step()
        p = r.plan
        trace = p.zeros(K, p.nchains, p.nspec, p.maxbins)
        r.capture_steps(K, trace=trace, trace_capacity=K, time_sweeps=True, time_every=every)
        if mode == "upload":
            ex = r.graph.raw_cuda_graph_exec()
            rc = hip.hipGraphUpload(ctypes.c_void_p(ex), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
            torch.cuda.synchronize()
            print("hipGraphUpload rc", rc)
        ts = [timed(r.step) / K * 1e3 for _ in range(4)]
        p.sweep_timing(False)
        print(mode, " ".join(f"{t:8.2f}" for t in ts), "us/step per replay")


if __name__ == "__main__":
    main(*sys.argv[1:])
