import ctypes, os, sys, torch
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "store_bw.so"))
n = 32 * 3 * 1025 * 1025
out = torch.empty(n + 64, dtype=torch.float64, device="cuda")
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
names = {0: "vec16 aligned", 1: "pair 8B", 2: "vec16 misaligned", 3: "row pattern"}
for grid in (2048, 8192, 32768):
    for which in (0, 1, 2, 3):
        for nt in (0, 1):
            ts = []
            for r in range(6):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(); lib.run(which, nt, ctypes.c_void_p(out.data_ptr()), ctypes.c_longlong(n), grid, s); e1.record()
                torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
            t = sorted(ts[1:])[len(ts[1:]) // 2]
            print(f"grid {grid:6d} {names[which]:18s} nt={nt}  {t*1e3:8.1f} us  {n*8/(t*1e-3)/1e9:7.1f} GB/s")
