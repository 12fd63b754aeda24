"""Time gs_nc_mh (propose + fused phases) at the bench size for several builds."""
import os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gibbssampler_amd import _capi as C
from gibbssampler_amd.problem import synthetic_problem
import gibbssampler_amd.engine as E
L, F, nch = 1024, 3, 32
P = synthetic_problem(L, 512, F, seed=0)
plans = []
for path in sys.argv[1:]:
    C._lib = None; C.load(path)
    p = E.GibbsPlan(L, 512, F, nch, P["bl"], P["noise_var"], P["bins"], blocks=P["blocks"], proposal_variances=P["proposal_variances"])
    p.lib = C._lib
    d = p.data_tensor(P["d_alm"]); dl = p.dl_tensor(P["dls_init"])
    _, st = p.cr_sweep(d, p.block_params(1, dl), seed=1, iteration=1)
    plans.append((path, p, st, dl))
res = {k[0]: [] for k in plans}
for rnd in range(6):
    for path, p, st, dl in plans:
        acc = p.zeros(nch, p.nacc, dtype=torch.int32)
        dd = dl.clone()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for it in range(10):
            p.nc_mh(st, dd, seed=3, iteration=it, accept=acc)
        e1.record(); torch.cuda.synchronize()
        if rnd: res[path].append(e0.elapsed_time(e1) / 10)
for k, v in res.items():
    print(f"{os.path.basename(k):30s} {np.median(v)*1e3:8.1f} us")
