"""Store-only replica of the CR sweep (tools/microbench/sweep_store.hip): GB/s of
the off-diagonal output stream for several field / chain strides."""
import ctypes, os
import numpy as np, torch
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), os.environ.get("SO", "sweep_store.so")))
import sys
L, nch = 1024, 32

NR = (L + 1) ** 2
def build(tm):
    # tasks: (tile group, chunk), heaviest first, dealt over 8 XCD buckets (as the plan)
    ntile = (L + 64) // 64
    work = []
    for g in range((ntile + 3) // 4):
        for c in range(0, (L - 256 * g) // tm + 1):
            wl = 0
            for t in range(4 * g, min(4 * g + 4, ntile)):
                lhi = L - 64 * t; lo = max(lhi - 63, 0)
                for m in range(c * tm, min(c * tm + tm, lhi + 1)):
                    wl += lhi - max(lo, m) + 1
            work.append((wl, g, c))
    work.sort(key=lambda w: -w[0])
    per = (len(work) + 7) // 8
    buckets = [[] for _ in range(8)]; load = [0] * 8
    for w in work:
        best = min((x for x in range(8) if len(buckets[x]) < per), key=lambda x: load[x])
        buckets[best].append((w[1], w[2])); load[best] += w[0]
    tasks = []
    for b in buckets:
        tasks += b + [(-1, 0)] * (per - len(b))
    tt = torch.tensor(tasks, dtype=torch.int32, device="cuda")
    # bytes written: off-diagonal blocks only (count on the host)
    nbytes = 0
    for (g, c) in tasks:
        if g < 0: continue
        for t in range(4 * g, min(4 * g + 4, ntile)):
            lhi = L - 64 * t; m0 = c * tm; m1 = min(m0 + tm, lhi + 1); lo = lhi - 63
            if m0 >= m1 or lo < 0 or m1 - 1 > lo: continue
            nbytes += (m1 - max(m0, 1)) * 64 * 16 * 3
    nbytes *= nch
    return tt, tasks, nbytes

big = torch.empty(3 * 300_000_000 // 8 * 8 + 32 * 3 * NR, dtype=torch.float64, device="cuda")
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
ntile = (L + 64) // 64


def build_rows_order(tm):
    """per-workgroup (g, c, chain): chunks dealt heaviest-first over 8 XCD buckets,
    inside a bucket chunk by chunk, chain by chain, the chunk's tile groups adjacent"""
    chunks = []
    for c in range(L // tm + 1):
        wl = 0; gs = []
        for g in range((ntile + 3) // 4):
            if c * tm <= L - 256 * g:
                gs.append(g)
                for t in range(4 * g, min(4 * g + 4, ntile)):
                    lhi = L - 64 * t; lo = max(lhi - 63, 0)
                    for m in range(c * tm, min(c * tm + tm, lhi + 1)):
                        wl += lhi - max(lo, m) + 1
        chunks.append((wl, c, gs))
    chunks.sort(key=lambda w: -w[0])
    buckets = [[] for _ in range(8)]; load = [0] * 8
    for w in chunks:
        b = min(range(8), key=lambda x: load[x]); buckets[b].append(w); load[b] += w[0]
    per = max(sum(len(w[2]) for w in b) for b in buckets) * nch
    items = []
    for b in buckets:
        lst = [(g, w[1], ch) for w in sorted(b, key=lambda w: w[1]) for ch in range(nch) for g in w[2]]
        lst += [(-1, 0, 0)] * (per - len(lst))
        items += lst
    return items


def time_rows_order(tm):
    items = build_rows_order(tm)
    tt = torch.tensor(items, dtype=torch.int32, device="cuda")
    _, _, nbytes = build(tm)
    ts = []
    for r in range(8):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        lib.run(L, nch, tm, ctypes.c_void_p(tt.data_ptr()), len(items), ctypes.c_void_p(big.data_ptr()),
                ctypes.c_longlong(NR), ctypes.c_longlong(3 * NR), 8, 0, s)
        e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
    t = sorted(ts[1:])[len(ts[1:]) // 2]
    print(f"tm {tm:3d} groups-adjacent order  {t*1e3:8.1f} us  {nbytes / (t * 1e-3) / 1e9:7.1f} GB/s", flush=True)


def timeit(tm, mode, grid=0, fs=NR, cs=3 * NR):
    tt, tasks, nbytes = build(tm)
    ts = []
    for r in range(8):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        lib.run(L, nch, tm, ctypes.c_void_p(tt.data_ptr()), len(tasks), ctypes.c_void_p(big.data_ptr()),
                ctypes.c_longlong(fs), ctypes.c_longlong(cs), mode, grid, s)
        e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
    t = sorted(ts[1:])[len(ts[1:]) // 2]
    print(f"tm {tm:3d} mode {mode} grid {grid:6d}  {t*1e3:8.1f} us  {nbytes / (t * 1e-3) / 1e9:7.1f} GB/s  ({nbytes/1e6:.0f} MB)",
          flush=True)


timeit(24, 0)
timeit(24, 6)
time_rows_order(24)
def time_rows(tm, align):
    nbytes = 16 * 3 * nch * sum(L + 1 - m for m in range(1, L + 1))
    ts = []
    for r in range(8):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        lib.run_rows(L, nch, tm, ctypes.c_void_p(big.data_ptr()), align, s)
        e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
    t = sorted(ts[1:])[len(ts[1:]) // 2]
    print(f"full rows align {align} tm {tm:3d}  {t*1e3:8.1f} us  {nbytes / (t * 1e-3) / 1e9:7.1f} GB/s", flush=True)


time_rows(24, 0)
time_rows(24, 2)
time_rows(8, 2)
time_rows(48, 2)
