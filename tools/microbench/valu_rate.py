"""Cycles per wave-instruction (per SIMD) of a few VALU ops on gfx950 (2.4 GHz assumed)."""
import ctypes, os, torch
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "valu_rate.so"))
nblk, n = 256 * 16, 4096
out = torch.empty(nblk * 256, dtype=torch.int64, device="cuda")
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
names = {0: "v_mad_u64_u32 (+ add)", 1: "v_fma_f64", 2: "v_mul_lo_u32 (+ add)", 3: "v_bitop3_b32"}
for op in (0, 1, 2, 3):
    ts = []
    for r in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); lib.run(op, ctypes.c_void_p(out.data_ptr()), nblk, n, s); e1.record()
        torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
    t = sorted(ts[1:])[len(ts[1:]) // 2] * 1e-3
    waves = nblk * 4
    instr_per_simd = waves * n * 8 / 1024
    print(f"{names[op]:24s} {t*1e3:8.2f} ms  {t * 2.4e9 / instr_per_simd:6.2f} cycles per wave-op-group", flush=True)
