"""Phase timeline of the fused MH kernel from a GS_MH_STAMPS build (s_memrealtime,
100 MHz): python tools/mh_stamps.py build_variants/lib_STAMPS.so"""
import ctypes, os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gibbssampler_amd import _capi as C
from gibbssampler_amd.problem import synthetic_problem
import gibbssampler_amd.engine as E
L, F, nch = 1024, 3, 32
P = synthetic_problem(L, 512, F, seed=0)
C.load(sys.argv[1])
p = E.GibbsPlan(L, 512, F, nch, P["bl"], P["noise_var"], P["bins"], blocks=P["blocks"],
                proposal_variances=P["proposal_variances"])
d = p.data_tensor(P["d_alm"]); dl = p.dl_tensor(P["dls_init"])
_, st = p.cr_sweep(d, p.block_params(1, dl), seed=1, iteration=1)
acc = p.zeros(nch, p.nacc, dtype=torch.int32)
buf = (ctypes.c_ulonglong * (64 * 24))()
rows = []
for it in range(12):
    p.nc_mh(st, dl, seed=3, iteration=it, accept=acc)
    torch.cuda.synchronize()
    C._lib.gs_debug_mh_stamps(buf)
    a = np.frombuffer(buf, dtype=np.uint64).reshape(64, 24)[:nch].astype(np.int64)
    if it >= 2:
        rows.append(a)
a = np.stack(rows)                     # [it, chain, 24]
t0 = a[:, :, 0:1]
rel = (a - t0) * 10.0 / 1000.0         # us
names = {1: "init done", 2: "ph0 terms", 3: "ph0 uniforms", 4: "ph0 narrow", 6: "ph0 wide / ph1 start",
         7: "ph1 terms", 8: "ph1 uniforms", 9: "ph1 narrow", 11: "ph1 wide / ph2 start", 12: "ph2 terms",
         13: "ph2 uniforms", 14: "ph2 narrow", 20: "phases done", 21: "writeback done"}
for k, n in names.items():
    v = rel[:, :, k]
    if np.all(a[:, :, k] == 0):
        continue
    print(f"{n:24s} median {np.median(v):7.2f} us  max {np.max(v):7.2f} us")
starts = (a[:, :, 0] - a[:, :, 0].min(axis=1, keepdims=True)) * 10.0 / 1000.0
print(f"workgroup start spread: median {np.median(starts.max(axis=1)):.2f} us")
