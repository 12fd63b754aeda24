"""Stage timeline of the MH kernel (k_mh_reg) from the "timeline" build variant
(build.py timeline -> libgibbs_hip_timeline.so, -DGS_MH_TIMELINE): thread 0 of
chain 0 stamps s_memrealtime (100 MHz) at the stage boundaries.

usage (GPU box, after `python gibbssampler_amd/build.py timeline` here):
  GIBBS_HIP_LIB=gibbssampler_amd/libgibbs_hip_timeline.so python tools/mh_timeline.py [L NSIDE NCHAINS]"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gibbssampler_amd import _capi  # noqa: E402
from gibbssampler_amd.problem import synthetic_problem  # noqa: E402
from gibbssampler_amd.samplers import BatchedRunner  # noqa: E402

NAMES = {0: "start", 1: "loads+LDS fill", 20: "D_l write-back"}
for q in range(4):
    NAMES[2 + 4 * q] = f"phase {q} terms"
    NAMES[3 + 4 * q] = f"phase {q} narrow"
    NAMES[4 + 4 * q] = f"phase {q} wide"
    NAMES[5 + 4 * q] = f"phase {q} barrier"


def main(L=1024, nside=512, nch=32):
    L, nside, nch = int(L), int(nside), int(nch)
    P = synthetic_problem(L, nside, 3, seed=0)
    r = BatchedRunner("noncentered", P["lmax"], P["nside"], 3, nch, P["bl"], P["noise_var"], P["bins"], P["d_alm"],
                      blocks=P["blocks"], proposal_variances=P["proposal_variances"], rng="native", seed=5)
    r.init(P["dls_init"])
    lib = _capi.load()
    fn = lib.gs_debug_mh_timeline
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    fn.restype = ctypes.c_int
    rows = []
    for it in range(12):
        r.step()
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * 32)()
        assert fn(buf) == 0
        t = np.array(buf[:], dtype=np.int64)
        if it >= 2:
            rows.append(t)
    rows = np.array(rows)
    t0 = rows[:, 0:1]
    rel = (rows - t0) * 10e-3      # 100 MHz ticks -> us
    med = np.median(rel, axis=0)
    prev = 0.0
    for k in sorted(NAMES):
        if np.all(rows[:, k] == 0):
            continue
        print(f"{NAMES[k]:20s} at {med[k]:7.2f} us  (+{med[k] - prev:6.2f})")
        prev = med[k]


if __name__ == "__main__":
    main(*sys.argv[1:])
