"""Turn gpurun_out/prof_<tag> rocprofv3 outputs (tools/profile_round.sh) into
committed profiles/ files.

  profiles/<tag>_kernel_stats.csv      rocprofv3 --stats summary of bench.py (default line)
  profiles/<tag>_<v>_pmc.csv           per-dispatch FETCH_SIZE / WRITE_SIZE of k_cr_sweep, variant <v>
  profiles/<tag>_<v>_valu.csv          per-dispatch VALU counters of k_cr_sweep, variant <v>
  profiles/<tag>_<mode>_kernel_stats.csv   kernel stats of configs[1], masked C5 / ASIS, SHT 2048
  profiles/pmc_traffic.json            per-launch HBM bytes and VALU work read by bench.py
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

# bench variant (tools/profile_round.sh) -> bench.py's profile key
VARIANTS = {
    "default": ("noncentered_L1024_F3_c32_nostore", "k_cr_sweep (STORE=false)"),
    "store": ("noncentered_L1024_F3_c32", "k_cr_sweep"),
    "c2": ("centered_L512_F3_c1_nostore", "k_cr_sweep (STORE=false, latency form)"),
    "c4": ("asis_L1024_F3_c32_nostore", "k_cr_sweep (STORE=false)"),
}


def counters(path):
    """{(dispatch, counter): value summed over the CSV's rows}"""
    cnt = {}
    for x in csv.DictReader(open(path)):
        k = (x["Dispatch_Id"], x["Counter_Name"])
        cnt[k] = cnt.get(k, 0.0) + float(x["Counter_Value"])
    return cnt


def per_dispatch(cnt, name):
    return [v for (d, n), v in sorted(cnt.items()) if n == name]


def variant(tag, src, dst, v, key, kernel, prof):
    d = os.path.join(src, v)
    fw = [os.path.join(d, k, "run_counter_collection.csv") for k in ("fetch", "write")]
    if not all(os.path.exists(p) for p in fw):
        print(f"{v}: no FETCH/WRITE pass, skipped")
        return
    rows, vals = [], {}
    for p in fw:
        for x in csv.DictReader(open(p)):
            rows.append({"counter": x["Counter_Name"], "dispatch": x["Dispatch_Id"], "kernel": x["Kernel_Name"][:40],
                         "value_kb": x["Counter_Value"]})
        for (_, n), val in counters(p).items():
            vals.setdefault(n, []).append(val)
    with open(os.path.join(dst, f"{tag}_{v}_pmc.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["counter", "dispatch", "kernel", "value_kb"])
        w.writeheader()
        w.writerows(rows)
    fetch = statistics.median(vals["FETCH_SIZE"]) * 1024 * 2.0
    write = statistics.median(vals["WRITE_SIZE"]) * 1024 * 1.0
    e = {"hbm_bytes_per_launch": int(fetch + write), "read_bytes": int(fetch), "write_bytes": int(write),
         "correction": "FETCH_SIZE x2, WRITE_SIZE x1 (calibrated: tools/microbench/calib.py)",
         "source": f"profiles/{tag}_{v}_pmc.csv", "kernel": kernel}
    valu = os.path.join(d, "valu", "run_counter_collection.csv")
    if os.path.exists(valu):
        cnt = counters(valu)
        fr, cyc = [], []
        for disp in sorted({k[0] for k in cnt}):
            # GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md DVFS note);
            # VALUBusy (derived_counters.xml) = SQ_ACTIVE_INST_VALU x 4 / (SIMDs x cycles);
            # gfx950 reports no SQ_INST_CYCLES_VALU
            c = cnt.get((disp, "GRBM_GUI_ACTIVE"), 0.0) / 8.0
            a = cnt.get((disp, "SQ_ACTIVE_INST_VALU"), 0.0) * 4.0
            if c > 0:
                fr.append(a / (1024.0 * c))
                cyc.append(a)
        if fr:
            e["valu_issue_frac"] = round(statistics.median(fr), 4)
            e["valu_busy_simd_cycles_per_launch"] = int(statistics.median(cyc))
            e["valu_insts_per_launch"] = int(statistics.median(per_dispatch(cnt, "SQ_INSTS_VALU")))
            e["valu_source"] = (f"profiles/{tag}_{v}_valu.csv: SQ_ACTIVE_INST_VALU x 4 = SIMD-busy cycles per "
                                f"launch; VALUBusy = that / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs)")
            shutil.copy(valu, os.path.join(dst, f"{tag}_{v}_valu.csv"))
    prof[key] = e
    print(f"{v:8s} {key:36s} {e}")


def main(tag="r03"):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    path = os.path.join(dst, "pmc_traffic.json")
    prof = json.load(open(path)) if os.path.exists(path) else {}
    for v, (key, kernel) in VARIANTS.items():
        variant(tag, src, dst, v, key, kernel, prof)
    json.dump(prof, open(path, "w"), indent=1)
    stats = {"": os.path.join(src, "trace", "run_kernel_stats.csv")}
    for mode in ("c2", "masked", "masked_asis", "sht"):
        stats["_" + mode] = os.path.join(f"{src}_{mode}", "run_kernel_stats.csv")
    for suffix, p in stats.items():
        if not os.path.exists(p):
            continue
        out = os.path.join(dst, f"{tag}{suffix}_kernel_stats.csv")
        shutil.copy(p, out)
        st = list(csv.DictReader(open(out)))
        print(f"\n{out}\n{'kernel':60s} {'calls':>6s} {'avg us':>9s} {'%':>6s}")
        for x in st[:12]:
            print(f"{x['Name'][:60]:60s} {x['Calls']:>6s} {float(x['AverageNs'])/1e3:9.2f} "
                  f"{float(x['Percentage']):6.2f}")


if __name__ == "__main__":
    main(*sys.argv[1:])
