"""Cycles per wave-instruction (per SIMD) of the CR sweep's VALU instruction
classes on gfx950, at 1 / 2 / 4 / 8 waves per SIMD (valu_rate.hip).

usage: python tools/microbench/valu_rate.py [--json out.json]
(build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o valu_rate.so valu_rate.hip)

Per op and waves-per-SIMD W: 256 x W workgroups of 4 waves; each wave stamps
s_memtime / s_memrealtime around its loop and its hardware slot, and the host
groups the waves by SIMD: cpi = (last end - first start on the SIMD) / (waves on
the SIMD x instructions per wave), median over the SIMDs.  The shader clock of
the run is memtime ticks / realtime ticks x 100 MHz.  Numbers in
profiles/r06_valu_rate.json; DESIGN.md section 3 weights the sweep loop's class
counts by them (tools/sweep_issue_model.py)."""
import argparse
import ctypes
import json
import os
import subprocess

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "valu_rate.so")
OPS = ["v_fma_f64", "v_mul_f64", "v_add_f64", "v_max_f64+v_min_f64 (fmin)", "v_mad_u64_u32", "v_bitop3_b32",
       "v_add_u32", "v_xor_b32", "v_lshrrev_b32", "v_cndmask_b32", "v_alignbit_b32", "v_bfe_u32", "v_med3_i32",
       "v_lshlrev_b64", "v_cvt_f64_u32", "v_cvt_i32_f64", "v_ldexp_f64", "v_frexp_mant_f64", "v_rsq_f64",
       "v_mul_lo_u32",
       "mix v_fma_f64 + v_bitop3_b32", "mix v_fma_f64 + v_add_u32", "mix v_fma_f64 + v_mad_u64_u32",
       "mix v_bitop3_b32 + v_mad_u64_u32", "mix v_fma_f64 + v_cvt_f64_u32"]
# VALU instructions per chain and step (the pairs issue two, fmin two)
PER = {3: 2, 20: 2, 21: 2, 22: 2, 23: 2, 24: 2}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--waves", default="1,2,4,8")
    a = ap.parse_args()
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(os.path.join(HERE, "valu_rate.hip")):
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-shared", "-fPIC", "-o", SO,
                        os.path.join(HERE, "valu_rate.hip")], check=True)
    lib = ctypes.CDLL(SO)
    lib.valu_rate_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_void_p]
    lib.valu_rate_run.restype = ctypes.c_int
    nops = lib.valu_rate_nops()
    assert nops == len(OPS), (nops, len(OPS))
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    res = {}
    for op in range(nops):
        res[OPS[op]] = {}
        for W in [int(w) for w in a.waves.split(",")]:
            nblk = 256 * W
            n = 1024 if W <= 2 else 512
            rec = torch.zeros(nblk * 4 * 6, dtype=torch.int64, device="cuda")
            sink = torch.zeros(nblk * 256, dtype=torch.int64, device="cuda")
            best = None
            for rep in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                rc = lib.valu_rate_run(op, rec.data_ptr(), sink.data_ptr(), nblk, n, st)
                e1.record()
                torch.cuda.synchronize()
                assert rc == 0, rc
                r = rec.view(-1, 6).cpu().numpy().astype(np.uint64)
                t0, t1, r0, r1, hw, xcc = (r[:, i] for i in range(6))
                simd = (hw >> 4) & 3
                cu = (hw >> 8) & 15
                sh = (hw >> 12) & 1
                se = (hw >> 13) & 7
                key = ((xcc & 15) << 12) | (se << 6) | (sh << 5) | (cu << 2) | simd
                ninstr = 2 * n * 8 * PER.get(op, 1)
                cpis = []
                for k in np.unique(key):
                    sel = key == k
                    el = float(t1[sel].max() - t0[sel].min())
                    cpis.append(el / (sel.sum() * ninstr))
                clk = float(np.median((t1 - t0).astype(np.float64) / (r1 - r0).astype(np.float64))) * 0.1  # GHz
                cur = {"cycles_per_instr": round(float(np.median(cpis)), 3),
                       "cpi_p10_p90": [round(float(np.percentile(cpis, 10)), 3),
                                       round(float(np.percentile(cpis, 90)), 3)],
                       "simds": int(len(cpis)), "clock_ghz": round(clk, 3),
                       "event_ms": round(e0.elapsed_time(e1), 4)}
                if best is None or cur["event_ms"] < best["event_ms"]:
                    best = cur
            res[OPS[op]][f"w{W}"] = best
            print(f"{OPS[op]:36s} W={W}: {best['cycles_per_instr']:6.2f} cyc/instr/SIMD  "
                  f"(p10-p90 {best['cpi_p10_p90']}, {best['simds']} SIMDs, {best['clock_ghz']:.2f} GHz, "
                  f"{best['event_ms']:.3f} ms)", flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"source": "tools/microbench/valu_rate.py (valu_rate.hip), MI355X gfx950",
                       "unit": "shader-clock cycles per wave64 instruction per SIMD; pairs: per instruction of the pair",
                       "device": torch.cuda.get_device_name(0), "ops": res}, f, indent=1)


if __name__ == "__main__":
    main()
