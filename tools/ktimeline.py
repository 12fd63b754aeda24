"""Print a window of a rocprofv3 kernel trace as a timeline (start / end in us
relative to the window, queue id, grid, short kernel name), to see whether
kernels of different streams overlap: python tools/ktimeline.py <dir> [--skip N] [--n M]"""
import csv
import re
import sys

d = sys.argv[1].rstrip("/")
skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 0
n = int(sys.argv[sys.argv.index("--n") + 1]) if "--n" in sys.argv else 60
rows = list(csv.DictReader(open(d + "/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[skip:skip + n]
t0 = int(rows[0]["Start_Timestamp"])
qcol = next((c for c in ("Queue_Id", "Stream_Id") if c in rows[0]), None)
print("columns:", ",".join(rows[0].keys()))
for r in rows:
    name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])
    name = re.sub(r"\((?!.*<).*$", "", name)[:40]
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    print(f"{s:10.1f} {e:10.1f} {e - s:8.1f}  q={r.get(qcol, '?'):>4s} s={r.get('Stream_Id', '?'):>4s} "
          f"{r['Grid_Size_X']:>8s}  {name}")
