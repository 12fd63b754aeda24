"""Fold the FETCH_SIZE / WRITE_SIZE passes of tools/step_traffic.py into
profiles/pmc_traffic.json: HBM bytes of ONE masked bench step (the dispatches
between the two k_remove_md markers), FETCH_SIZE x2 (the calibrated gfx950 read
correction, tools/microbench/calib.py) + WRITE_SIZE x1, both KB per dispatch
summed over the XCDs (MI355X_MICROARCH.md rocprofv3 section), with the top
kernels and the ratio to the step's algorithmic bytes (every transform reads its
input and writes its output once: 8 ncomp ((L+1)^2 + Npix) bytes per map and
transform, bench.py's SHT count per step).

usage: python tools/summarize_step_traffic.py <fetch_dir> <write_dir> <log>
(<log>: tools/step_traffic.py's output, whose STEP_TRAFFIC line names the
workload and its SHT count; the record goes to pmc_traffic.json key
step_<workload>_N<nside>_L<lmax>_B<nchains>_<mask>)
"""
import collections
import csv
import json
import os
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def window(path, counter):
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    marks = [i for i, r in enumerate(rows) if "k_remove_md" in r["Kernel_Name"]]
    if len(marks) < 2:
        raise SystemExit(f"{path}: markers not found ({len(marks)})")
    per = collections.defaultdict(float)
    for r in rows[marks[-2] + 1:marks[-1]]:
        per[r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]] += float(r["Counter_Value"])
    return per


def main():
    fdir, wdir, log = sys.argv[1:4]
    meta = json.loads(next(l for l in open(log) if l.startswith("STEP_TRAFFIC "))[len("STEP_TRAFFIC "):])
    n_sht, B, ncomp, N, L = float(meta["n_sht"]), meta["nchains"], meta["ncomp"], meta["nside"], meta["lmax"]
    key = f"step_{meta['workload']}_N{N}_L{L}_B{B}_{meta['mask']}"
    f = window(os.path.join(fdir, "run_counter_collection.csv"), "FETCH_SIZE")
    w = window(os.path.join(wdir, "run_counter_collection.csv"), "WRITE_SIZE")
    per = {k: 2 * 1024 * f.get(k, 0.0) + 1024 * w.get(k, 0.0) for k in set(f) | set(w)}
    total = sum(per.values())
    alg = n_sht * 8 * ncomp * ((L + 1) ** 2 + 12 * N * N) * B
    tag = "r06_" + key
    dst = {}
    for d, c in ((fdir, "fetch"), (wdir, "write")):
        out = os.path.join(ROOT, "profiles", f"{tag}_{c}.csv")
        shutil.copy(os.path.join(d, "run_counter_collection.csv"), out)
        dst[c] = os.path.relpath(out, ROOT)
    top = sorted(per.items(), key=lambda kv: -kv[1])[:8]
    rec = {"hbm_bytes_per_step": int(total), "algorithmic_bytes_per_step": int(alg),
           "traffic_over_algorithmic": round(total / alg, 3),
           "top_kernels_bytes": {k: int(v) for k, v in top},
           "source": f"{dst['fetch']} / {dst['write']} (FETCH_SIZE x2 + WRITE_SIZE, KB x 1024, the dispatches of "
                     f"one bench step between the tools/step_traffic.py markers)",
           "algorithmic_note": f"{n_sht} SHT-equivalents x 8 B x {ncomp} comps x ((L+1)^2 + Npix) x {B} chains"}
    pj = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    data = json.load(open(pj)) if os.path.exists(pj) else {}
    data[key] = rec
    json.dump(data, open(pj, "w"), indent=1)
    print(key, json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
