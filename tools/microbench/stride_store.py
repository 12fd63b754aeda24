"""GB/s of a 768 MB write stream vs the distance between a wave's consecutive 1-KB stores."""
import ctypes, os, torch
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "stride_store.so"))
lib.run.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
lib.run.restype = ctypes.c_int
nkb = 768 * 1024
out = torch.empty(nkb * 128, dtype=torch.float64, device="cuda")
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
for nt in (1, 0):
    for R in (24, 72):
        for G in (1, 2, 4, 8, 16, 64, 256):
            nw = (nkb // R) // (4 * G) * (4 * G)
            ts = []
            for r in range(6):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                assert (nw * R) * 128 <= out.numel(), (nw, R)
                e0.record(); rc = lib.run(out.data_ptr(), nw * R, R, G, nt, s.value); e1.record()
                assert rc == 0, f"launch error {rc}"
                torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
            t = sorted(ts[1:])[len(ts[1:]) // 2]
            print(f"nt {nt} R {R:3d} G {G:4d}  {t*1e3:8.1f} us  {nw*R*1024/(t*1e-3)/1e9:7.1f} GB/s", flush=True)
