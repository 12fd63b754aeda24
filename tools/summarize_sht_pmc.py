"""Fold tools/profile_round.sh part c (r04) into profiles/: per-kernel HBM bytes,
achieved bandwidth and wave-state fractions of the chain-batched SHT (N_side
256, 16 spin-2 maps, matrix-core Legendre tables) and of the N_side 2048
recurrence kernels, plus the per-map transform traffic that bench.py's masked
lines report as roofline.traffic (profiles/pmc_traffic.json key
masked_sht_N256_L512_B16).

usage: python tools/summarize_sht_pmc.py <tag>   (reads gpurun_out/prof_<tag>_shtb, _sht2048)

Units and corrections (MI355X_MICROARCH.md, rocprofv3 section): FETCH_SIZE and
WRITE_SIZE are KB per dispatch summed over the XCDs; FETCH_SIZE x2 (the
calibrated gfx950 read correction, tools/microbench/calib.py), WRITE_SIZE x1;
SQ_* wave counters count quad-cycles, SQ_VALU_MFMA_BUSY_CYCLES counts cycles;
GRBM_GUI_ACTIVE is summed over the 8 XCDs.
"""
import collections
import csv
import json
import os
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
NSIMD = 1024


def counters(path):
    """kernel -> counter -> list of per-dispatch values"""
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    if not os.path.exists(path):
        return out
    for r in csv.DictReader(open(path)):
        out[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return out


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0]


def durations(path):
    out = {}
    if not os.path.exists(path):
        return out
    for r in csv.DictReader(open(path)):
        out[short(r["Name"])] = (float(r["AverageNs"]) * 1e-9, int(r["Calls"]))
    return out


def mean(v):
    return sum(v) / len(v) if v else None


def summarize(base, dur):
    f = counters(os.path.join(base, "fetch_size", "run_counter_collection.csv"))
    w = counters(os.path.join(base, "write_size", "run_counter_collection.csv"))
    q = counters(os.path.join(base, "sq_wave_cycles", "run_counter_collection.csv"))
    if not q:
        q = counters(os.path.join(base, "sq_insts_valu", "run_counter_collection.csv"))
    res = {}
    for k in sorted(set(f) | set(w) | set(q)):
        e = {}
        rd = mean(f[k].get("FETCH_SIZE", [])) if k in f else None
        wr = mean(w[k].get("WRITE_SIZE", [])) if k in w else None
        if rd is not None:
            e["read_bytes"] = int(rd * 1024 * 2)
        if wr is not None:
            e["write_bytes"] = int(wr * 1024)
        if rd is not None and wr is not None:
            e["hbm_bytes"] = e["read_bytes"] + e["write_bytes"]
        d = dur.get(k)
        if d:
            e["avg_s"] = d[0]
            if "hbm_bytes" in e:
                e["hbm_GBps"] = round(e["hbm_bytes"] / d[0] / 1e9, 1)
        if k in q:
            c = {n: mean(v) for n, v in q[k].items()}
            grbm = c.get("GRBM_GUI_ACTIVE")
            if grbm:
                cyc = grbm / 8.0                      # per XCD = kernel cycles
                e["kernel_cycles"] = int(cyc)
                if c.get("SQ_VALU_MFMA_BUSY_CYCLES") is not None:
                    e["mfma_busy_frac"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (NSIMD * cyc), 4)
                if c.get("SQ_ACTIVE_INST_VALU") is not None:
                    e["valu_busy_frac"] = round(4 * c["SQ_ACTIVE_INST_VALU"] / (NSIMD * cyc), 4)
            wc = c.get("SQ_WAVE_CYCLES")
            if wc:
                for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                    if c.get(n) is not None:
                        e[n.lower() + "_frac"] = round(c[n] / wc, 4)
            for n in ("SQ_INSTS_MFMA", "SQ_INSTS_VALU"):
                if c.get(n) is not None:
                    e[n.lower()] = int(c[n])
        res[k] = e
    return res


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r04"
    out = {}
    b = os.path.join(ROOT, "gpurun_out", f"prof_{tag}_shtb")
    dur = durations(os.path.join(b, "trace", "run_kernel_stats.csv"))
    out["sht_N256_L512_B16_spin2_mfma"] = summarize(b, dur)
    ba = os.path.join(ROOT, "gpurun_out", f"prof_{tag}_shta")
    if os.path.isdir(ba):
        out["sht_N256_L512_B16_spin2_apply_band"] = summarize(ba, durations(os.path.join(ba, "trace",
                                                                                        "run_kernel_stats.csv")))
    b2 = os.path.join(ROOT, "gpurun_out", f"prof_{tag}_sht2048")
    out["sht_N2048_L4096_TEB_recurrence"] = summarize(b2, durations(os.path.join(ROOT, "profiles",
                                                                                 "r03_sht_kernel_stats.csv")))
    dst = os.path.join(ROOT, "profiles", f"{tag}_sht_pmc.json")
    json.dump(out, open(dst, "w"), indent=1)
    print("wrote", dst)
    for name, sub in (("shtb", b), ("shta", ba), ("sht2048", b2)):
        for d in ("fetch_size", "write_size", "sq_wave_cycles", "sq_insts_valu"):
            src = os.path.join(sub, d, "run_counter_collection.csv")
            if os.path.exists(src):
                shutil.copy(src, os.path.join(ROOT, "profiles", f"{tag}_{name}_{d}.csv"))
        src = os.path.join(sub, "trace", "run_kernel_stats.csv")
        if os.path.exists(src):
            shutil.copy(src, os.path.join(ROOT, "profiles", f"{tag}_{name}_kernel_stats.csv"))
    # per-map bytes of one transform (16-map batch), for bench.py's masked lines
    s = out["sht_N256_L512_B16_spin2_mfma"]
    syn = [k for k in s if ("synth" in k or "alm_in" in k) and "hbm_bytes" in s[k]]
    ana = [k for k in s if "anal" in k and "hbm_bytes" in s[k]]
    if syn and ana:
        a2m = sum(s[k]["hbm_bytes"] for k in syn) / 16
        m2a = sum(s[k]["hbm_bytes"] for k in ana) / 16
        p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        j = json.load(open(p))
        j["masked_sht_N256_L512_B16"] = {
            "alm2map_bytes_per_map": int(a2m), "map2alm_bytes_per_map": int(m2a),
            "bytes_per_transform_per_map": int((a2m + m2a) / 2),
            "kernels": {"alm2map": syn, "map2alm": ana},
            "correction": "FETCH_SIZE x2, WRITE_SIZE x1 (calibrated: tools/microbench/calib.py)",
            "source": f"profiles/{tag}_shtb_fetch_size.csv, profiles/{tag}_shtb_write_size.csv "
                      "(tools/sht_bench.py --nside 256 --batch 16 --ncomp 2 --mfma)"}
        json.dump(j, open(p, "w"), indent=1)
        print("pmc_traffic.json: alm2map %.1f MB, map2alm %.1f MB per map" % (a2m / 1e6, m2a / 1e6))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
