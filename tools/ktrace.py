"""Group a rocprofv3 kernel trace by (kernel, grid) and, optionally, restrict it to
the last N steps' window: python tools/ktrace.py <dir> [--since-frac F]
Prints calls, mean and total microseconds per (short kernel name, grid)."""
import csv
import re
import sys
from collections import defaultdict

d = sys.argv[1].rstrip("/")
rows = list(csv.DictReader(open(d + "/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
frac = float(sys.argv[sys.argv.index("--since-frac") + 1]) if "--since-frac" in sys.argv else 0.0
t0, t1 = int(rows[0]["Start_Timestamp"]), int(rows[-1]["End_Timestamp"])
cut = t0 + frac * (t1 - t0)
agg = defaultdict(lambda: [0, 0.0])
for r in rows:
    if int(r["Start_Timestamp"]) < cut:
        continue
    name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
    name = re.sub(r"\((?!.*<).*$", "", name)[:48]
    key = (name, r["Grid_Size_X"] + "x" + r["Grid_Size_Y"])
    a = agg[key]
    a[0] += 1
    a[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
tot = sum(v[1] for v in agg.values())
for (n, g), (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
    print(f"{n:48s} {g:>14s} {c:6d} {t / c:10.1f} us {t / 1e3:9.2f} ms {100 * t / tot:5.1f}%")
print(f"total {tot / 1e3:.2f} ms")
