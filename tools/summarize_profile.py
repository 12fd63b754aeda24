"""Turn gpurun_out/prof_<tag> rocprofv3 outputs into committed profiles/ files.

  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats summary of bench.py
  profiles/<tag>_pmc.csv            per-dispatch FETCH_SIZE / WRITE_SIZE of k_cr_sweep
  profiles/pmc_traffic.json         HBM bytes per sweep launch read by bench.py
The FETCH_SIZE correction (x2) and WRITE_SIZE (x1) were calibrated on gfx950
with the sweep's own 8-byte lane-pair access shape (tools/microbench/calib.py):
FETCH_SIZE read 0.500x and WRITE_SIZE 1.003x of 1 GiB of known traffic.
"""
import csv
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(tag="r02", key="noncentered_L1024_F3_c32"):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, f"{tag}_kernel_stats.csv"))
    rows, vals = [], {}
    for kind in ("fetch", "write"):
        for x in csv.DictReader(open(os.path.join(src, kind, "run_counter_collection.csv"))):
            rows.append({"counter": x["Counter_Name"], "dispatch": x["Dispatch_Id"], "kernel": x["Kernel_Name"][:40],
                         "value_kb": x["Counter_Value"]})
            vals.setdefault(x["Counter_Name"], []).append(float(x["Counter_Value"]))
    with open(os.path.join(dst, f"{tag}_pmc.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["counter", "dispatch", "kernel", "value_kb"])
        w.writeheader()
        w.writerows(rows)
    fetch = statistics.median(vals["FETCH_SIZE"]) * 1024 * 2.0
    write = statistics.median(vals["WRITE_SIZE"]) * 1024 * 1.0
    path = os.path.join(dst, "pmc_traffic.json")
    prof = json.load(open(path)) if os.path.exists(path) else {}
    prof[key] = {"hbm_bytes_per_launch": int(fetch + write), "read_bytes": int(fetch), "write_bytes": int(write),
                 "correction": "FETCH_SIZE x2, WRITE_SIZE x1 (calibrated: tools/microbench/calib.py)",
                 "source": f"profiles/{tag}_pmc.csv", "kernel": "k_cr_sweep"}
    # VALU issue fraction of the sweep: SIMD cycles of VALU work / (SIMDs x cycles);
    # GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md DVFS note)
    valu_csv = os.path.join(src, "valu", "run_counter_collection.csv")
    if os.path.exists(valu_csv):
        cnt = {}
        for x in csv.DictReader(open(valu_csv)):
            cnt.setdefault((x["Dispatch_Id"], x["Counter_Name"]), 0.0)
            cnt[(x["Dispatch_Id"], x["Counter_Name"])] += float(x["Counter_Value"])
        fr = []
        for d in sorted({k[0] for k in cnt}):
            cyc = cnt.get((d, "GRBM_GUI_ACTIVE"), 0.0) / 8.0
            if cyc > 0:
                # VALUBusy (derived_counters.xml) with GRBM_GUI_ACTIVE per XCD:
                # SQ_ACTIVE_INST_VALU x 4 / (SIMDs x cycles); gfx950 reports no
                # SQ_INST_CYCLES_VALU
                fr.append(cnt.get((d, "SQ_ACTIVE_INST_VALU"), 0.0) * 4.0 / (1024.0 * cyc))
        if fr:
            prof[key]["valu_issue_frac"] = round(statistics.median(fr), 4)
            prof[key]["valu_insts_per_launch"] = int(statistics.median(
                [v for (d, n), v in cnt.items() if n == "SQ_INSTS_VALU"]))
            prof[key]["valu_source"] = (f"profiles/{tag}_valu.csv: SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x "
                                        f"GRBM_GUI_ACTIVE / 8 XCDs) (VALUBusy)")
            shutil.copy(valu_csv, os.path.join(dst, f"{tag}_valu.csv"))
    json.dump(prof, open(path, "w"), indent=1)
    # summary table
    st = list(csv.DictReader(open(os.path.join(dst, f"{tag}_kernel_stats.csv"))))
    print(f"{'kernel':60s} {'calls':>6s} {'avg us':>9s} {'%':>6s}")
    for x in st:
        print(f"{x['Name'][:60]:60s} {x['Calls']:>6s} {float(x['AverageNs'])/1e3:9.2f} {float(x['Percentage']):6.2f}")
    print("traffic per sweep launch (bytes):", prof[key])


if __name__ == "__main__":
    main(*sys.argv[1:])
