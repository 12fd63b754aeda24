"""Time the CR sweep (+ statistics finish) for several rows-per-task settings in
one process (interleaved rounds; GS_SWEEP_ROWS is read at plan creation).

usage (GPU box): python tools/sweep_rows.py 16 32 64 ..."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gibbssampler_amd.problem import synthetic_problem  # noqa: E402
import gibbssampler_amd.engine as E  # noqa: E402


def main():
    rows = [int(a) for a in sys.argv[1:]] or [32]
    L, nside, F, nch = int(os.environ.get("L", 1024)), 512, 3, int(os.environ.get("NCH", 32))
    P = synthetic_problem(L, nside, F, seed=0)
    plans = []
    for tm in rows:
        os.environ["GS_SWEEP_ROWS"] = str(tm)
        p = E.GibbsPlan(L, nside, F, nch, P["bl"], P["noise_var"], P["bins"], blocks=P["blocks"],
                        proposal_variances=P["proposal_variances"])
        plans.append(p)
    d = plans[0].data_tensor(P["d_alm"])
    outs = []
    for p in plans:
        dl = p.dl_tensor(P["dls_init"])
        outs.append((p.block_params(1, dl), p.zeros(nch, F, p.NR), p.zeros(nch, p.nstat, L + 1)))
    times = {k: [] for k in range(len(plans))}
    for rnd in range(8):
        for k, p in enumerate(plans):
            params, s, st = outs[k]
            for _ in range(3):
                p.cr_sweep(d, params, seed=1, iteration=rnd, s_out=s, stats=st)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for it in range(20):
                p.cr_sweep(d, params, seed=1, iteration=it, s_out=s, stats=st)
            e1.record()
            torch.cuda.synchronize()
            if rnd >= 1:
                times[k].append(e0.elapsed_time(e1) / 20)
    nbytes = 8 * F * (L + 1) ** 2 * (nch + 1)
    for k, tm in enumerate(rows):
        t = np.median(times[k])
        print(f"rows {tm:4d}  median {t*1e3:8.1f} us  min {min(times[k])*1e3:8.1f} us  "
              f"{nbytes / (t * 1e-3) / 1e9:7.1f} GB/s (sweep+finish)", flush=True)


if __name__ == "__main__":
    main()
