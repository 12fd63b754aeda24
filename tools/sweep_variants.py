"""Time the CR sweep at the bench configuration for several library builds.

usage (GPU box): python tools/sweep_variants.py lib1.so lib2.so ...
Interleaves the variants in one process (rounds x variants) and reports the
median launch time of gs_cr_sweep measured with hipEvents on the launch stream.
"""
import ctypes
import sys
import os

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gibbssampler_amd import _capi as C  # noqa: E402
from gibbssampler_amd.problem import synthetic_problem  # noqa: E402


STORE = os.environ.get('STORE', '1') == '1'


def main():
    libs = sys.argv[1:]
    L, nside, F, nch = int(os.environ.get("L", 1024)), 512, 3, int(os.environ.get("NCH", 32))
    P = synthetic_problem(L, nside, F, seed=0)
    import gibbssampler_amd.engine as E
    plans = []
    for path in libs:
        C._lib = None
        C.load(path)
        p = E.GibbsPlan(L, nside, F, nch, P["bl"], P["noise_var"], P["bins"], blocks=P["blocks"],
                        proposal_variances=P["proposal_variances"])
        p.lib = C._lib
        plans.append(p)
    d = plans[0].data_tensor(P["d_alm"])
    times = {k: [] for k in range(len(libs))}
    outs = []
    for p in plans:
        dl = p.dl_tensor(P["dls_init"])
        params = p.block_params(1, dl)
        s = p.zeros(nch, F, p.NR)
        st = p.zeros(nch, p.nstat, L + 1)
        outs.append((params, s, st))
    for rnd in range(7):
        for k, p in enumerate(plans):
            params, s, st = outs[k]
            for _ in range(3):
                p.cr_sweep(d, params, seed=1, iteration=rnd, s_out=s, stats=st, store=STORE)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for it in range(20):
                p.cr_sweep(d, params, seed=1, iteration=it, s_out=s, stats=st, store=STORE)
            e1.record()
            torch.cuda.synchronize()
            if rnd >= 1:
                times[k].append(e0.elapsed_time(e1) / 20)
    nbytes = 8 * F * (L + 1) ** 2 * (nch + 1)
    for k, path in enumerate(libs):
        t = np.median(times[k])
        print(f"{os.path.basename(path):40s} median {t*1e3:8.1f} us  min {min(times[k])*1e3:8.1f} us  "
              f"{nbytes / (t * 1e-3) / 1e9:7.1f} GB/s (sweep+finish)")


if __name__ == "__main__":
    main()
