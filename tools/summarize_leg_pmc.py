"""Per-kernel summary of tools/sht_pmc.sh's passes over the VALU Legendre kernels:
average duration (kernel trace), SIMD VALU busy, the wave-state fractions and
the scalar-load latency.

usage: python tools/summarize_leg_pmc.py gpurun_out/shtpmc_<tag> [--json out.json]

Units (MI355X_MICROARCH.md, rocprofv3 section): SQ_WAVE_CYCLES, SQ_WAIT_*,
SQ_ACTIVE_INST_* count quad-cycles per wave; GRBM_GUI_ACTIVE is summed over the
8 XCDs, so VALU busy = SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8);
SQ_INST_LEVEL_SMEM / SQ_INSTS_SMEM = the mean in-flight time of a scalar load.
"""
import argparse
import collections
import csv
import json
import os


def short(name):
    return name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]


def counters(path):
    """kernel -> counter -> mean per dispatch"""
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        per[(short(r["Kernel_Name"]), r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for (k, _), c in per.items():
        for n, v in c.items():
            out[k][n].append(v)
    return {k: {n: sum(v) / len(v) for n, v in c.items()} for k, c in out.items()}


def durations(path):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        d[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    st = counters(os.path.join(a.dir, "stall", "run_counter_collection.csv"))
    me = counters(os.path.join(a.dir, "mem", "run_counter_collection.csv"))
    dur = durations(os.path.join(a.dir, "trace", "run_kernel_trace.csv"))
    res = {}
    for k in sorted(st):
        s, m = st[k], me.get(k, {})
        wc = s.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        grbm = s.get("GRBM_GUI_ACTIVE", 0.0)
        ds = dur.get(k, [])
        r = {"dispatches_timed": len(ds),
             "avg_ms": round(sum(ds) / len(ds), 4) if ds else None,
             "valu_busy": round(s["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * grbm / 8), 4) if grbm else None,
             "wave_frac_valu": round(s.get("SQ_ACTIVE_INST_VALU", 0) / wc, 4),
             "wave_frac_wait_any": round(s.get("SQ_WAIT_ANY", 0) / wc, 4),
             "wave_frac_wait_issue": round(s.get("SQ_WAIT_INST_ANY", 0) / wc, 4),
             "waves_per_simd": round(s.get("SQ_WAVE_CYCLES", 0) * 4 / (1024 * grbm / 8), 3) if grbm else None,
             "smem_latency_cycles": round(m["SQ_INST_LEVEL_SMEM"] / m["SQ_INSTS_SMEM"], 1)
             if m.get("SQ_INSTS_SMEM") else None,
             "valu_instr": m.get("SQ_INSTS_VALU"), "smem_instr": m.get("SQ_INSTS_SMEM"),
             "lds_instr": m.get("SQ_INSTS_LDS"),
             "lds_bank_conflict_frac": round(m["SQ_LDS_BANK_CONFLICT"] / m["SQ_ACTIVE_INST_LDS"], 4)
             if m.get("SQ_ACTIVE_INST_LDS") else None}
        res[k] = r
        print(k, json.dumps(r))
    if a.json:
        json.dump(res, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
