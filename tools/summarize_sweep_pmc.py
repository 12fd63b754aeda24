"""Fold tools/sweep_pmc.sh's passes (gpurun_out/pmc_<tag>/) over the headline
sweep into profiles/: the per-dispatch counter files and the
noncentered_L1024_F3_c32_nostore record of profiles/pmc_traffic.json that
bench.py's roofline quotes (SIMD-busy cycles, VALU busy at the run clock, the
hardware's VALU class counts, the dual-issue fraction, HBM bytes).

usage: python tools/summarize_sweep_pmc.py <tag>

Units (MI355X_MICROARCH.md, rocprofv3 section): SQ_ACTIVE_INST_VALU counts
quad-cycles (x4 = SIMD-busy cycles), GRBM_GUI_ACTIVE is summed over the 8 XCDs
(VALU busy = SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8));
FETCH_SIZE x2 (the calibrated gfx950 read correction, tools/microbench/calib.py)
and WRITE_SIZE x1, KB per dispatch summed over the XCDs.
"""
import csv
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEY = "noncentered_L1024_F3_c32_nostore"


def per_dispatch(path):
    """dispatch -> counter -> value (summed over the CSV's rows)"""
    out = {}
    for r in csv.DictReader(open(path)):
        if "k_cr_sweep" not in r["Kernel_Name"]:
            continue
        d = out.setdefault(int(r["Dispatch_Id"]), {})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def med(dd, name, f=lambda c: c):
    vals = [f(c) for c in dd.values() if name in c]
    return statistics.median(vals) if vals else None


def main(tag):
    src = os.path.join(ROOT, "gpurun_out", f"pmc_{tag}")
    dst = os.path.join(ROOT, "profiles")
    st = per_dispatch(os.path.join(src, "stall", "run_counter_collection.csv"))
    cl = per_dispatch(os.path.join(src, "cls", "run_counter_collection.csv"))
    fe = per_dispatch(os.path.join(src, "fetch", "run_counter_collection.csv"))
    wr = per_dispatch(os.path.join(src, "write", "run_counter_collection.csv"))
    files = {"valu": ("stall", f"{tag}_default_valu.csv"), "valu_classes": ("cls", f"{tag}_default_valu_classes.csv")}
    for _, (d, name) in files.items():
        shutil.copy(os.path.join(src, d, "run_counter_collection.csv"), os.path.join(dst, name))
    with open(os.path.join(dst, f"{tag}_default_pmc.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["counter", "dispatch", "kernel", "value_kb"])
        for name, dd in (("FETCH_SIZE", fe), ("WRITE_SIZE", wr)):
            for disp, c in sorted(dd.items()):
                w.writerow([name, disp, "k_cr_sweep<3, 0, false, 0>", c.get(name)])
    ts = os.path.join(src, "trace", "run_kernel_stats.csv")
    if os.path.exists(ts):
        shutil.copy(ts, os.path.join(dst, f"{tag}_kernel_stats.csv"))
    busy = med(st, "SQ_ACTIVE_INST_VALU", lambda c: c["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * c["GRBM_GUI_ACTIVE"] / 8))
    cyc = med(st, "SQ_ACTIVE_INST_VALU", lambda c: c["SQ_ACTIVE_INST_VALU"] * 4)
    insts = med(st, "SQ_INSTS_VALU", lambda c: c["SQ_INSTS_VALU"])
    fetch = med(fe, "FETCH_SIZE", lambda c: c["FETCH_SIZE"]) * 1024 * 2.0
    write = med(wr, "WRITE_SIZE", lambda c: c["WRITE_SIZE"]) * 1024 * 1.0
    dual = med(cl, "SQ_ACTIVE_INST_VALU2", lambda c: c["SQ_ACTIVE_INST_VALU2"])
    classes = {n: int(med(cl, n, lambda c, n=n: c[n])) for n in sorted({k for c in cl.values() for k in c})
               if n.startswith("SQ_INSTS_VALU_")}
    path = os.path.join(dst, "pmc_traffic.json")
    prof = json.load(open(path))
    prof[KEY] = {
        "hbm_bytes_per_launch": int(fetch + write), "read_bytes": int(fetch), "write_bytes": int(write),
        "correction": "FETCH_SIZE x2, WRITE_SIZE x1 (calibrated: tools/microbench/calib.py)",
        "source": f"profiles/{tag}_default_pmc.csv", "kernel": "k_cr_sweep (STORE=false)",
        "valu_issue_frac": round(busy, 4), "valu_busy_simd_cycles_per_launch": int(cyc),
        "valu_insts_per_launch": int(insts),
        "valu_source": f"profiles/{tag}_default_valu.csv: SQ_ACTIVE_INST_VALU x 4 = SIMD-busy cycles per launch; "
                       f"VALUBusy = that / (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs)",
        "dual_issue_quad_cycles_per_launch": int(dual) if dual is not None else None,
        "dual_issue_frac": round(dual * 4 / cyc, 4) if dual is not None else None,
        "valu_classes_per_launch": classes,
        "classes_source": f"profiles/{tag}_default_valu_classes.csv (SQ_INSTS_VALU_* and SQ_ACTIVE_INST_VALU2: "
                          f"quad-cycles with two VALU instructions issued)"}
    json.dump(prof, open(path, "w"), indent=1)
    print(json.dumps(prof[KEY], indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
