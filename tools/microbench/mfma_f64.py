"""Cycles per v_mfma_f64_16x16x4_f64 per SIMD on gfx950 (clock 2.4 GHz assumed),
alone and with 8 independent v_fma_f64 of the same wave per MFMA."""
import ctypes, os, subprocess, torch
here = os.path.dirname(os.path.abspath(__file__))
so = os.path.join(here, "mfma_f64.so")
lib = ctypes.CDLL(so)
nblk, n = 256 * 8, 2048
out = torch.empty(nblk * 256, dtype=torch.float64, device="cuda")
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
for mode in (0, 1):
    ts = []
    for r in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); lib.run(mode, ctypes.c_void_p(out.data_ptr()), nblk, n, s); e1.record()
        torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
    t = sorted(ts[1:])[len(ts[1:]) // 2] * 1e-3
    mfma_per_simd = nblk * 4 * n * 4 / 1024
    cyc = t * 2.4e9 / mfma_per_simd
    print(f"mode {mode}: {t*1e3:8.3f} ms, {cyc:6.2f} cycles per MFMA per SIMD, "
          f"{nblk * 4 * n * 4 * 2048 / t / 1e12:6.2f} TF/s", flush=True)
