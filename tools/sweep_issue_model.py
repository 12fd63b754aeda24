"""The headline CR sweep's issue ceiling from a MEASURED instruction-class mix
(VERDICT r05 item 1): the gfx950 ISA of k_cr_sweep<3,0,false,0>'s row loop
(hipcc -S of the product source, the loop that holds the three Philox calls),
each VALU opcode weighted by its measured cycles per wave-instruction at 8
waves per SIMD (tools/microbench/valu_rate.py -> profiles/r06_valu_rate.json),
times the wave-rows of one configs[2] launch (32 chains, L 1024: every (tile,
row) of the triangle once per chain).  Writes profiles/r06_sweep_issue_model.json,
which bench.py's roofline quotes next to the PMC-counted SIMD-busy cycles.

usage: python tools/sweep_issue_model.py [--valu-rate profiles/r06_valu_rate.json]
"""
import argparse
import collections
import json
import os
import re
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
KERNEL = r"_Z10k_cr_sweepILi3ELi0ELb0ELi0EE"

# opcode (prefix) -> the microbench class whose W=8 rate prices it
CLASS = [
    (r"v_(fma|fmac|mul|add)_f64", "v_fma_f64"),
    (r"v_(min|max)_f64", "v_max_f64+v_min_f64 (fmin)"),
    (r"v_ldexp_f64", "v_ldexp_f64"),
    (r"v_frexp_(mant|exp_i32)_f64", "v_frexp_mant_f64"),
    (r"v_cvt_f64_(u32|i32)", "v_cvt_f64_u32"),
    (r"v_cvt_i32_f64", "v_cvt_i32_f64"),
    (r"v_rsq_f64", "v_rsq_f64"),
    (r"v_cmp_\w+_f64", "v_fma_f64"),
    (r"v_mad_u64_u32", "v_mad_u64_u32"),
    (r"v_bitop3_b32", "v_bitop3_b32"),
    (r"v_(add|sub|subrev)_u32|v_(xor|or|and)_b32", "v_add_u32"),
    (r"v_(lshrrev|lshlrev)_b32", "v_lshrrev_b32"),
    (r"v_lshl_add_u64|v_lshlrev_b64", "v_lshlrev_b64"),
    (r"v_cndmask_b32", "v_lshrrev_b32"),
    (r"v_alignbit_b32", "v_alignbit_b32"),
    (r"v_bfe_u32", "v_bfe_u32"),
    (r"v_med3_i32", "v_med3_i32"),
    (r"v_mov_b(32|64)|v_cmp_\w+_[iu]32|v_subbrev_co_u32", "v_add_u32"),
]


def loop_hist(asm):
    s = open(asm).read().split("\n")
    k = [i for i, l in enumerate(s) if re.match(r"^" + KERNEL + r"\S*:", l)][0]
    en = [i for i in range(k, len(s)) if s[i].strip().startswith("s_endpgm")][0]
    body = s[k:en]
    labels = {m.group(1): i for i, l in enumerate(body) for m in [re.match(r"^(\.LBB\S+):", l)] if m}
    best = None
    for i, l in enumerate(body):
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\S+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            c = collections.Counter()
            for x in body[labels[m.group(1)]:i + 1]:
                x = x.strip()
                if x and not x.startswith((".", ";")) and not x.endswith(":"):
                    c[x.split()[0]] += 1
            # the row loop: three Philox calls (>= 40 v_mad_u64_u32), the
            # off-diagonal form (no per-lane row test: the fewest instructions)
            if c["v_mad_u64_u32"] >= 40 and (best is None or sum(c.values()) < sum(best.values())):
                best = c
    return best


def wave_rows(L=1024, nchains=32, tile=64):
    """every (tile, row m <= l_hi) of the triangle, once per chain"""
    return nchains * sum(L - tile * t + 1 for t in range((L + tile) // tile) if L - tile * t >= 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--valu-rate", default=os.path.join(ROOT, "profiles", "r06_valu_rate.json"))
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r06_sweep_issue_model.json"))
    a = ap.parse_args()
    raw = {k: v["w8"]["cycles_per_instr"] for k, v in json.load(open(a.valu_rate))["ops"].items()}
    # the microbench loop (16 instructions of the class, a counter, a compare and
    # a taken branch per iteration) adds a fixed issue overhead per instruction;
    # it is calibrated out with v_fma_f64, whose rate is fixed by the part's
    # fp64 peak (78.6 TF/s = 1024 SIMDs x 2.4 GHz x 16 FMA lanes: 4 cycles per
    # wave64 instruction)
    ovh = raw["v_fma_f64"] - 4.0
    rates = {k: round(v - ovh, 3) for k, v in raw.items()}
    with tempfile.TemporaryDirectory() as td:
        asm = os.path.join(td, "k.s")
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-ffp-contract=on", "-std=c++17", "-I",
                        os.path.join(ROOT, "include"), "--cuda-device-only", "-S", "-o", asm,
                        os.path.join(ROOT, "gibbssampler_amd", "csrc", "gs_kernels.hip")], check=True,
                       stderr=subprocess.DEVNULL)
        hist = loop_hist(asm)
    valu, other, priced = 0, {}, collections.defaultdict(lambda: [0, 0.0])
    cyc = 0.0
    for op, n in hist.items():
        if not op.startswith("v_"):
            other[op] = n
            continue
        cls = next((c for pat, c in CLASS if re.match(pat, op)), None)
        if cls is None:
            raise SystemExit(f"unpriced VALU opcode {op}")
        valu += n
        priced[cls][0] += n
        priced[cls][1] += n * rates[cls]
        cyc += n * rates[cls]
    wr = wave_rows()
    out = {"kernel": "k_cr_sweep<3,0,false,0> row loop (gfx950 ISA of the product source)",
           "valu_instructions_per_row": valu, "non_valu_per_row": other,
           "classes": {k: {"count": v[0], "cycles": round(v[1], 1), "cycles_per_instr": rates[k], "measured_w8": raw[k]}
                       for k, v in sorted(priced.items(), key=lambda kv: -kv[1][1])},
           "issue_cycles_per_row": round(cyc, 1),
           "microbench_loop_overhead_per_instr": round(ovh, 3),
           "flat4_cycles_per_row": 4 * valu,
           "wave_rows_per_launch": wr,
           "issue_cycles_per_simd": round(cyc * wr / 1024, 0),
           "floor_us_at_2p4GHz": round(cyc * wr / 1024 / 2.4e3, 2),
           "source": "tools/sweep_issue_model.py: ISA class counts x profiles/r06_valu_rate.json (W = 8 rates less "
                     "the microbench loop's overhead per instruction, calibrated on v_fma_f64 = 4 cycles)"}
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
