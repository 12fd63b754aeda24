#!/usr/bin/env python
"""Gibbs iterations/sec on MI355X -- BASELINE.json metric.

Workload (default, BASELINE.json configs[2]): NonCenteredGibbs TEB, all_sph
full sky, N_side = 512, l_max = 1024, 32 chains per GPU, synthetic data
(SURVEY.md 8d fiducial), native Philox RNG.  One "step" = one Gibbs
iteration (constrained realisation + C_l draw) of every chain on every GPU.

  python bench.py [--gpus N --steps K --warmup W --workload NAME]

  noncentered          configs[2] (default line)
  centered             configs[1] shape (--lmax 512 --nside 256 --nchains 1)
  asis                 configs[3] per GPU (32 chains / GPU)
  masked               configs[4]: centered TEB, 80% mask, aux CR n_gibbs 1, N_side 2048 / L 4096
  masked_centered_ula  HEAD's main_polarization.py run (:113-115,154): masked CenteredGibbs,
                       gibbs_cr + ula (aux + MALA), EB, N_side 256 / L 512, 1 chain / GPU
  masked_asis          HEAD's ASIS (:121-124): masked, all_sph=False, gibbs_cr, over-relaxation,
                       n_gibbs 20, pixel-domain MH (f2), EB, N_side 256 / L 512, 1 chain / GPU
  masked_centered_pcg  HEAD's centered_gibbs (:109-111): masked, gibbs_cr=False, ula=False -> the
                       PCG CR (f1, device-resident CG) every iteration + C_l draw, EB, N256 / L512
  masked_noncentered   HEAD's non_centered_gibbs (:117-120) with the mask: PCG CR, C^-1/2, the
                       pixel-domain MH sweep (f2), EB, N_side 256 / L 512, 1 chain / GPU

For N > 1 launch with torch.distributed.run (one rank per GPU, RCCL): chains
are sharded (global chain id = rank * chains_per_gpu + c) by
gibbssampler_amd.distributed.ShardContext, no collective runs inside an
iteration; the D_l traces are all-gathered once after the timed region.
value = total chain-iterations / max-over-ranks wall time.
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: 8.0 TB/s spec
FP64_VALU_PEAK_TFS = 78.6    # MI355X_MICROARCH.md: FP64 vector
VALU_SIMDS = 1024            # 256 CUs x 4 SIMDs
VALU_CLOCK_GHZ = 2.4         # peak engine clock
METRIC = "Gibbs iters/sec (constrained-realization + C_l draw), Nside=%d lmax=%d"
HARMONIC = ("noncentered", "centered", "asis")
SURFACE = ("surface_noncentered",)
MASKED_HEAD = ("masked_centered_ula", "masked_asis", "masked_centered_pcg", "masked_noncentered")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed steps (500; masked: 50; HEAD modes: 5)")
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--workload", default="noncentered",
                    choices=list(HARMONIC) + ["masked"] + list(MASKED_HEAD) + list(SURFACE))
    ap.add_argument("--nchains", type=int, default=None, help="chains per GPU (32; masked: 1)")
    ap.add_argument("--lmax", type=int, default=None, help="1024 (masked: 4096; HEAD modes: 512)")
    ap.add_argument("--nside", type=int, default=None, help="512 (masked: 2048; HEAD modes: 256)")
    ap.add_argument("--fields", type=int, default=3, choices=[1, 2, 3])
    ap.add_argument("--seed", type=int, default=20261015)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=10.0, help="seconds per CPU baseline leg")
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of one hipGraph of the timed steps")
    ap.add_argument("--time-every", type=int, default=None,
                    help="bracket the CR sweep of every N-th timed step with hipEvents (graph mode); each "
                         "event pair is an extra pair of graph nodes in its step, so sampling every 10th "
                         "sweep keeps the timed steps close to the un-instrumented graph (default: 10, or "
                         "steps // 5 for runs under 100 steps: the driver's 20-step command samples 5 sweeps)")
    ap.add_argument("--mask", default="band", choices=["band", "galactic"],
                    help="masked workloads: SURVEY 8d's |cos theta| > 0.2 band, or data.galactic_mask (wavy edge)")
    ap.add_argument("--skymap", default="none", choices=["store", "none"],
                    help="harmonic workloads: 'none' (default) runs the CR sweep without writing the sky map s -- "
                         "a full-sky run never reads it: the next CR, the MH and the C_l draw use the per-l "
                         "statistics only, and the reference's run() returns D_l and accept flags only "
                         "(NonCenteredGibbs.py:529-571); 'store' writes s every iteration (HBM roofline)")
    ap.add_argument("--ramp-ms", type=float, default=None,
                    help="harmonic modes: milliseconds of the same workload on a scratch runner (other chains, "
                         "untimed) before the warmup steps, so a short timed region (e.g. --steps 20) is not "
                         "measured while the GPU's clocks still ramp up (clock_ramp); reported in the line "
                         "(default 200; 0 turns it off)")
    ap.add_argument("--profile-json", default=os.path.join(HERE, "profiles", "pmc_traffic.json"))
    ap.add_argument("--opt", action="append", default=[],
                    help="NAME=VALUE library option (gs_option_set, include/gibbs_capi.h) set before any plan is made "
                         "(A/B of a plan choice; the line's config records it)")
    a = ap.parse_args()
    one = a.workload == "masked" or a.workload in MASKED_HEAD
    a.nchains = a.nchains or (1 if one else 32)
    if a.workload in MASKED_HEAD:
        a.lmax, a.nside = a.lmax or 512, a.nside or 256
        a.steps, a.warmup = a.steps or 5, a.warmup if a.warmup is not None else 1
    else:
        a.lmax = a.lmax or (4096 if a.workload == "masked" else 1024)
        a.nside = a.nside or (2048 if a.workload == "masked" else 512)
        # harmonic modes: 500 timed steps (a timed region of ~0.1 s, past the GPU's
        # clock ramp; the reference's runs are 10^4 iterations), 20 warmup steps
        harmonic = a.workload != "masked"
        a.steps = a.steps or (500 if harmonic else 50)
        a.warmup = a.warmup if a.warmup is not None else (20 if harmonic else 5)
    a.ramp_ms = a.ramp_ms if a.ramp_ms is not None else 200.0
    if a.time_every is None:
        # every event pair costs its step ~0.1 % (measured: the driver's 20-step
        # command timing all 20 sweeps ran 0.1937 against 0.1916 ms per step
        # timing 2, with the same sweep average, profiles/r06u_*): 10 for long
        # runs, >= 5 samples for short ones
        a.time_every = 10 if a.steps >= 100 else max(1, a.steps // 5)
    return a


def clock_ramp(args, make_runner, ms):
    """Bring the GPU to its steady clocks before the warmup: a scratch runner of
    the same workload (its own chains -- seed + 1 -- and buffers; the measured
    runner is not touched) replays a captured 20-step graph for `ms`
    milliseconds, untimed.  Measured (r05, 20 timed steps after 5 warmup steps,
    as the driver runs bench.py): no ramp 0.277-0.285 ms/step, 300 ms of fp64
    GEMM 0.248-0.252, 300 ms of fp64 elementwise work 0.246, 100 / 300 ms of this
    ramp 0.237 / 0.2345 -- the 500-step steady state (0.2345-0.241): the clocks
    ramp on this workload's own instruction mix (VALU-bound), not on any load.
    Returns the milliseconds spent and the scratch runner, which the caller
    drops after the timed region (its teardown frees device memory: host time
    with the GPU idle, which must not fall between the ramp and the warmup)."""
    import torch
    if ms <= 0:
        return 0.0, None
    scratch = make_runner(args.seed + 1)
    g = scratch.capture_steps(20)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        g.replay()
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3, scratch


def sweep_algorithmic_bytes(L, F, nchains, store=True):
    """Unique HBM bytes one CR-sweep launch must move (DESIGN.md 'Roofline'):
    write s (8 F (L+1)^2 per chain; none with --skymap none) + read the shared
    data once (8 F (L+1)^2) + read the per-l operator table (80 B per chain and
    l).  The per-task statistics partials are implementation traffic and are
    not counted."""
    NR = (L + 1) ** 2
    return (8 * F * NR * nchains if store else 0) + 8 * F * NR + 80 * (L + 1) * nchains


def sweep_roofline(args, prof, alg_bytes, achieved, sweep_avg_ms, sweep_n, one_graph):
    """The dominant kernel's roofline.  With the sky map stored (--skymap store)
    the sweep is bounded by HBM: unique bytes (write s, read d once, the operator)
    per launch / the launch's measured duration.  Without the store the sweep
    moves ~83 MB per launch and is bounded by VALU issue: the SIMD-busy cycles
    one launch needs (SQ_ACTIVE_INST_VALU x 4, counted by the profile pass for
    this kernel and configuration, profiles/pmc_traffic.json) / the launch's
    measured duration, against 1024 SIMDs x the 2.4 GHz peak engine clock."""
    timing = ("hipEvents around each sweep inside the timed graph" if one_graph else
              "hipEvents around each sweep of the timed loop")
    common = {"avg_launch_ms": round(sweep_avg_ms, 5), "launches": sweep_n, "timing": timing,
              "traffic": prof.get("hbm_bytes_per_launch"), "algorithmic_bytes_per_launch": alg_bytes}
    if args.skymap == "store":
        return {"bound": "hbm", "kernel": "k_cr_sweep", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), **common,
                "valu_issue_frac": prof.get("valu_issue_frac"),
                "note": "the sweep is close to issue-bound as well (Philox + Box-Muller per normal, DESIGN.md 3): "
                        "valu_issue_frac = SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8) from "
                        "the profile pass (profiles/pmc_traffic.json)"}
    # the issue ceiling from the MEASURED instruction-class mix (VERDICT r05 item 1;
    # tools/sweep_issue_model.py): the loop's VALU opcodes from the ISA, each
    # priced at its measured cycles per wave-instruction (8 waves per SIMD,
    # tools/microbench/valu_rate.py), x the launch's wave-rows: the rate at which
    # 1024 SIMDs at the 2.4 GHz peak clock could issue rows of this mix
    model = {}
    try:
        with open(os.path.join(HERE, "profiles", "r06_sweep_issue_model.json")) as f:
            model = json.load(f)
    except (OSError, ValueError):
        pass
    if model and args.lmax == 1024 and args.nchains == 32 and args.fields == 3:
        rows = model["wave_rows_per_launch"]
        cpr = model["issue_cycles_per_row"]
        ach = rows / (sweep_avg_ms * 1e-3) / 1e9
        peak = VALU_SIMDS * VALU_CLOCK_GHZ / cpr
        cyc = prof.get("valu_busy_simd_cycles_per_launch")
        return {"bound": "valu", "kernel": "k_cr_sweep (sky map not stored)",
                "achieved": round(ach, 4), "peak": round(peak, 4), "unit": "G wave-rows/s",
                "frac": round(ach / peak, 4), **common,
                "issue_model": {"wave_rows_per_launch": rows, "issue_cycles_per_row": cpr,
                                "valu_instructions_per_row": model["valu_instructions_per_row"],
                                "class_cycles_per_row": {k: v["cycles"] for k, v in model["classes"].items()},
                                "class_cycles_per_instr": {k: v["cycles_per_instr"] for k, v in model["classes"].items()},
                                "microbench_loop_overhead_per_instr": model.get("microbench_loop_overhead_per_instr"),
                                "source": "profiles/r06_sweep_issue_model.json (tools/sweep_issue_model.py) x "
                                          "profiles/r06_valu_rate.json (tools/microbench/valu_rate.py)"},
                "pmc": {"valu_busy_simd_cycles_per_launch": cyc,
                        "valu_busy_frac_of_peak_clock": round(cyc / (VALU_SIMDS * VALU_CLOCK_GHZ * 1e9 *
                                                                     sweep_avg_ms * 1e-3), 4) if cyc else None,
                        "valu_busy_frac_at_run_clock": prof.get("valu_issue_frac"),
                        "dual_issue_frac": prof.get("dual_issue_frac"),
                        "source": prof.get("valu_source")},
                "hbm_frac_unique_bytes": round(achieved / HBM_PEAK_GBS, 4),
                "note": "issue-bound: Philox4x32-10 + fp64 Box-Muller per normal (DESIGN.md 3).  peak = 1024 SIMDs x "
                        "2.4 GHz / the mix-weighted cycles per wave-row; achieved = the launch's wave-rows / its "
                        "duration measured here (hipEvents in the timed graph).  Measured class costs (8 waves per "
                        "SIMD, the microbench loop's overhead calibrated out on v_fma_f64 = 4): fp64 and most 32-bit "
                        "VALU ~3.9-4.0, v_mad_u64_u32 4.2, v_bitop3 3.2, v_add/xor_u32 2.1 (they dual-issue only "
                        "beside each other: mixed with fp64 every op costs a quad-cycle; the launch's PMC "
                        "dual-issue fraction is pmc.dual_issue_frac), v_rsq_f64 16."}
    cyc = prof.get("valu_busy_simd_cycles_per_launch")
    peak = VALU_SIMDS * VALU_CLOCK_GHZ
    ach = cyc / (sweep_avg_ms * 1e-3) / 1e9 if cyc else None
    return {"bound": "valu", "kernel": "k_cr_sweep (sky map not stored)",
            "achieved": round(ach, 1) if ach else None, "peak": peak, "unit": "G SIMD-busy cycles/s",
            "frac": round(ach / peak, 4) if ach else None, **common,
            "valu_busy_simd_cycles_per_launch": cyc, "valu_issue_frac_at_run_clock": prof.get("valu_issue_frac"),
            "hbm_frac_unique_bytes": round(achieved / HBM_PEAK_GBS, 4),
            "note": "issue-bound: Philox4x32-10 + fp64 Box-Muller per normal (DESIGN.md 3); achieved = the launch's "
                    "SIMD-busy cycles (SQ_ACTIVE_INST_VALU x 4 from the profile pass of this kernel and config) / "
                    "its duration measured here; peak = 1024 SIMDs x 2.4 GHz"}


def sht_flops(nside, L, c):
    """N_ringpair * N_lm * c (c = 4 spin-0, 16 spin-2, 20 TEB)."""
    return 2 * nside * (L + 1) * (L + 2) // 2 * c


def load_profile(path, key):
    try:
        with open(path) as f:
            return json.load(f).get(key, {})
    except (OSError, ValueError):
        return {}


def cpu_baseline_child(args):
    """The CPU baselines on the host's cores (one chain per core, at most 32:
    one GPU's share of the 8-GPU node's 256 cores), run as a child process before this process
    touches the GPU: the reference-structured port and the algorithm-matched
    port (oracle/cpu_baseline.py)."""
    env = dict(os.environ, OMP_NUM_THREADS="1", OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "oracle.cpu_baseline", "--lmax", str(args.lmax), "--nside", str(args.nside),
           "--fields", str(args.fields), "--budget", str(args.cpu_budget)]
    try:
        out = subprocess.run(cmd, cwd=HERE, env=env, capture_output=True, text=True, timeout=300, check=True)
        r = json.loads(out.stdout.strip().splitlines()[-1])
    except (subprocess.SubprocessError, ValueError, IndexError) as e:
        print(f"cpu baseline failed: {e}", file=sys.stderr)
        return None
    cores = r["cores"]
    ref, mat = r["reference"], r["matched"]
    return {"value": round(ref["value"], 5), "unit": "chain-iterations/s", "cores": cores, "kind": "port",
            "sample": f"{ref['iterations']} NonCentered TEB all_sph iterations, one chain per core on {cores} cores "
                      f"(of {r['affinity']} in the affinity mask), Nside={args.nside} lmax={args.lmax}, "
                      f"{ref['seconds']:.1f} s wall: vectorised numpy port with the reference's per-block "
                      f"full-sky likelihood (oracle/cpu_baseline.py nc_iteration)",
            "algorithm_matched": {"value": round(mat["value"], 4), "unit": "chain-iterations/s", "cores": cores,
                                  "sample": f"{mat['iterations']} iterations in {mat['seconds']:.1f} s with the "
                                            f"GPU's per-l statistics (oracle/cpu_baseline.py nc_iteration_matched)"}}


def cpu_baseline_masked_child(args):
    """The masked workloads' CPU leg (oracle/cpu_baseline_masked.py: the reference's
    masked samplers with the C++/OpenMP HEALPix SHT of oracle/sht_cpu.cpp on
    min(affinity, 32) threads), run as a child process before this process
    touches the GPU; a PCG workload's rate is completed with the device solve's
    CG iteration count after the timed region (cpu_baseline_masked.finalize)."""
    env = dict(os.environ, OPENBLAS_NUM_THREADS="1", MKL_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "oracle.cpu_baseline_masked", "--workload", args.workload, "--nside", str(args.nside),
           "--lmax", str(args.lmax)]
    try:
        # stderr passes through: the child's progress lines keep a long CPU leg visible
        out = subprocess.run(cmd, cwd=HERE, env=env, stdout=subprocess.PIPE, text=True, timeout=900, check=True)
        return json.loads(out.stdout.strip().splitlines()[-1])
    except (subprocess.SubprocessError, ValueError, IndexError) as e:
        print(f"masked cpu baseline failed: {e}", file=sys.stderr)
        return None


def _finalize_cpu(cpu, cg_iters=None):
    if cpu is None:
        return None
    from oracle.cpu_baseline_masked import finalize
    return finalize(cpu, cg_iters)


def cpu_leg(args):
    """The CPU baseline of this workload (None when it has none)."""
    if args.no_cpu_baseline:
        return None
    if args.workload == "noncentered":
        return cpu_baseline_child(args)
    if args.workload == "masked" or args.workload in MASKED_HEAD:
        return cpu_baseline_masked_child(args)
    return None


def self_launch(args):
    """``bench.py --gpus N`` (N > 1) started without torchrun: the CPU baseline
    first (this process never touches the GPU), then N ranks of this script under
    torch.distributed.run (one per GPU, RCCL), rank 0's JSON line completed with
    the CPU baseline.  Exits non-zero when the ranks fail or report another GPU
    count -- one GPU is never measured in place of N."""
    from gibbssampler_amd.distributed import launch_ranks
    cpu = cpu_leg(args)
    argv = [a for a in sys.argv[1:]]
    if "--no-cpu-baseline" not in argv:
        argv.append("--no-cpu-baseline")
    try:
        # GS_BENCH_RANK_SCRIPT: a stand-in rank program (the CPU launcher test)
        script = os.environ.get("GS_BENCH_RANK_SCRIPT", os.path.abspath(__file__))
        line, _ = launch_ranks(args.gpus, script, argv, cwd=HERE)
    except Exception as e:            # noqa: BLE001 -- reported, then a non-zero exit
        print(f"bench.py --gpus {args.gpus}: the rank launch failed: {e}", file=sys.stderr)
        raise SystemExit(2)
    if line.get("n_gpus") != args.gpus:
        print(f"bench.py --gpus {args.gpus}: the ranks reported n_gpus={line.get('n_gpus')}", file=sys.stderr)
        raise SystemExit(2)
    return attach_cpu(line, cpu)


def attach_cpu(line, cpu):
    """rank 0's line + the CPU baseline measured before the ranks started (a PCG
    workload's CPU rate takes the device solve's CG iteration count)."""
    if cpu is not None and line.get("cpu_baseline") is None:
        if "seconds_per_iteration" in cpu:          # the masked legs' raw form
            pcg = line.get("pcg") or {}
            cpu = _finalize_cpu(cpu, pcg.get("cg_iterations_per_solve"))
        line["cpu_baseline"] = cpu
        line.setdefault("notes_cpu", "cpu_baseline measured by the launching process before the ranks started")
    return line


def main():
    args = parse()
    from gibbssampler_amd.distributed import ShardContext, dist_env
    world, rank, local = dist_env()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        print(json.dumps(self_launch(args)))
        return
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: launch one rank per GPU "
              f"(python -m torch.distributed.run --nproc-per-node {args.gpus} bench.py --gpus {args.gpus}, "
              f"or plain python bench.py --gpus {args.gpus})", file=sys.stderr)
        raise SystemExit(2)
    # under torchrun (N > 1) the CPU baseline is the launcher's (self_launch);
    # at N = 1 this process runs it before touching the GPU
    cpu = cpu_leg(args) if rank == 0 and world == 1 else None
    import torch
    torch.cuda.set_device(local)
    ctx = ShardContext(args.nchains, backend="nccl")
    from gibbssampler_amd.build import build
    if ctx.rank == 0:
        build()
    ctx.barrier()
    if args.opt:
        from gibbssampler_amd import _capi
        for o in args.opt:
            k, v = o.split("=", 1)
            _capi.set_option(k, v)
    try:
        if args.workload in HARMONIC:
            line = run_harmonic(args, ctx, cpu)
        elif args.workload in SURFACE:
            line = run_surface(args, ctx)
        elif args.workload == "masked":
            line = run_masked(args, ctx, cpu)
        else:
            line = run_masked_head(args, ctx, cpu)
        if ctx.rank == 0:
            if args.opt:
                line["config"]["library_options"] = dict(o.split("=", 1) for o in args.opt)
            print(json.dumps(line))
    finally:
        ctx.close()


def run_harmonic(args, ctx, cpu):
    import torch
    from gibbssampler_amd.problem import synthetic_problem
    from gibbssampler_amd.samplers import BatchedRunner

    P = synthetic_problem(args.lmax, args.nside, args.fields, seed=0)

    def make_runner(seed):
        r = BatchedRunner(kind=args.workload, lmax=P["lmax"], nside=P["nside"], nfields=P["nfields"],
                          nchains=args.nchains, bl=P["bl"], noise_var=P["noise_var"], bins=P["bins"],
                          d_alm=P["d_alm"], blocks=P["blocks"], proposal_variances=P["proposal_variances"],
                          rng="native", seed=seed, chain0=ctx.chain0, store_skymap=args.skymap == "store")
        r.init(P["dls_init"])
        return r

    runner = make_runner(args.seed)
    p = runner.plan
    trace = p.zeros(args.steps, p.nchains, p.nspec, p.maxbins)
    one_graph = not args.no_graph
    warm_graph = None
    ramp, scratch = 0.0, None
    if one_graph and args.warmup > 0:
        # the W warmup steps as one hipGraph, replayed right before the timed
        # replay (below): besides warming the kernels this pays the process's
        # one-time cost of its first graph launch (~1.9 ms at configs[2],
        # measured), and the GPU enters the timed region busy -- capturing the
        # timed graph after the warmup left the GPU idle for the capture's host
        # time, and the timed replay then ran ~5 % slower than later replays
        # (tools/replay_probe.py)
        warm_graph = runner.capture_steps(args.warmup)
    else:
        if not one_graph:
            ramp, scratch = clock_ramp(args, make_runner, args.ramp_ms)
        for _ in range(args.warmup):
            runner.step()
    if one_graph:
        # the K timed iterations as ONE hipGraph (D_l trace written on the device);
        # every CR-sweep kernel is bracketed by event-record nodes inside the graph,
        # so its duration is measured on its stream over the timed region itself
        runner.capture_steps(args.steps, trace=trace, trace_capacity=args.steps, time_sweeps=True,
                             time_every=args.time_every)
        # the GEMM ramp between the captures (host time, GPU idle) and the warmup
        # replay: the GPU enters the warmup and the timed steps at speed
        ramp, scratch = clock_ramp(args, make_runner, args.ramp_ms)
        if warm_graph is not None:
            warm_graph.replay()
            runner.iteration += args.warmup
    else:
        p.sweep_timing(True)
    torch.cuda.synchronize()
    ctx.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if one_graph:
        runner.step()                   # one replay = the K steps
    else:
        for i in range(args.steps):
            runner.step()
            trace[i].copy_(runner.dl)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    ctx.barrier()
    elapsed = ctx.max(t1 - t0)
    del scratch
    sweep_ms, sweep_n = p.sweep_timing(False)
    # the run's only collective: every rank's D_l traces, gathered over RCCL / xGMI
    gathered = ctx.gather(trace)
    torch.cuda.synchronize()
    assert gathered.shape[1] == ctx.global_chains
    if ctx.rank != 0:
        return None
    total = args.steps * ctx.global_chains
    sweep_avg_ms = sweep_ms / max(sweep_n, 1)
    alg_bytes = sweep_algorithmic_bytes(p.L, p.F, p.nchains, store=args.skymap == "store")
    achieved = alg_bytes / (sweep_avg_ms * 1e-3) / 1e9
    prof = load_profile(args.profile_json, f"{args.workload}_L{args.lmax}_F{args.fields}_c{p.nchains}"
                        + ("" if args.skymap == "store" else "_nostore"))
    return {
        "metric": METRIC % (args.nside, args.lmax),
        "value": round(total / elapsed, 3),
        "unit": "chain-iterations/s",
        "n_gpus": ctx.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (analytic fiducial spectra, d = b s + n in harmonic space, seed 0)",
        "config": {"workload": f"{args.workload} {'TEB' if args.fields == 3 else 'F=%d' % args.fields} all_sph "
                               f"full-sky" + (" (TEB semantics build-specified; the reference's HEAD is EB, "
                                              "parity for TT/TE pinned against the oracle only)"
                                              if args.fields == 3 else ""),
                   "launch": "one hipGraph of all timed iterations" if one_graph else "eager",
                   "skymap": "stored every iteration" if args.skymap == "store" else
                             "not stored (CR draw reduced to the per-l statistics in registers; s is never read "
                             "by a full-sky run)",
                   "nside": args.nside, "lmax": args.lmax, "nfields": args.fields,
                   "chains_per_gpu": args.nchains, "global_chains": ctx.global_chains,
                   "rng": "native philox4x32-10", "parallelism": f"chains sharded over {ctx.world} GPU(s)"},
        "roofline": sweep_roofline(args, prof, alg_bytes, achieved, sweep_avg_ms, sweep_n, one_graph),
        "cpu_baseline": cpu,
        "clock_ramp": {"ms": round(ramp, 1),
                       "work": "a scratch runner of this workload (seed + 1, its own buffers) replaying a 20-step "
                               "graph, untimed, before the warmup steps (bench.clock_ramp)"},
    }


def run_surface(args, ctx):
    """BASELINE configs[2] through the drop-in class surface a
    main_polarization.py caller uses (gibbs.NonCenteredGibbs, all_sph, TEB,
    native streams): wall time of ``run(dls_init)`` for --steps iterations --
    the runner's replays of captured hipGraph chunks (32 steps each), the
    per-chunk trace copies and the histories' transfer to the host included.
    An untimed run of the same --steps iterations first builds the plan and
    captures the chunk graphs (run() keeps them: a sampler's later runs replay
    them without capturing)."""
    import torch
    from gibbssampler_amd.gibbs import NonCenteredGibbs
    from gibbssampler_amd.problem import synthetic_problem
    L, N = args.lmax, args.nside
    P = synthetic_problem(L, N, 3, seed=0)
    d = P["d_alm"]
    pix = {"TT": d[0], "EE": d[1], "BB": d[2]}
    nv = P["noise_var"]
    ncg = NonCenteredGibbs(pix, float(nv[0]), float(nv[1]), 0.5, N, L, 12 * N * N, P["proposal_variances"],
                           metropolis_blocks=P["blocks"], polarization=True, bins=P["bins"], all_sph=True,
                           n_iter=args.steps, rng="native", seed=args.seed, nchains=args.nchains,
                           fields="TEB", chain0=ctx.chain0)
    ncg.run(P["dls_init"])
    torch.cuda.synchronize()
    ctx.barrier()
    t0 = time.perf_counter()
    out = ncg.run(P["dls_init"])
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    ctx.barrier()
    elapsed = ctx.max(t1 - t0)
    if ctx.rank != 0:
        return None
    hist = out[0]
    assert np.asarray(hist["EE"]).shape[0] == args.steps + 1
    total = args.steps * ctx.global_chains
    return {
        "metric": METRIC % (N, L), "value": round(total / elapsed, 3), "unit": "chain-iterations/s",
        "n_gpus": ctx.world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (analytic fiducial spectra, d = b s + n in harmonic space, seed 0)",
        "config": {"workload": "noncentered TEB all_sph full-sky through gibbs.NonCenteredGibbs.run (drop-in surface)",
                   "launch": "run(): replays of the sampler's captured 32-step hipGraph chunks, each chunk's histories to pinned host memory on a copy stream under the next chunk",
                   "nside": N, "lmax": L, "nfields": 3, "chains_per_gpu": args.nchains,
                   "global_chains": ctx.global_chains, "rng": "native philox4x32-10",
                   "parallelism": f"chains sharded over {ctx.world} GPU(s)"},
        "roofline": None, "cpu_baseline": None,
        "notes": "the surface's own throughput (VERDICT r01 item 10); the roofline of its sweep is the default line's",
    }


def _masked_data(N, L, nfields, seed=0, mask_kind="band"):
    """synfast of the fiducial spectra on the device + white noise + the 80%
    band mask (mask_kind "galactic": data.galactic_mask, a wavy
    galactic-plane cut whose edge crosses rings), as host arrays."""
    import torch
    from gibbssampler_amd.data import band_mask, galactic_mask, synfast
    from gibbssampler_amd.problem import fiducial_dl
    dl = fiducial_dl(L, 3)
    ell = np.arange(L + 1, dtype=np.float64)
    fac = np.where(ell > 0, 2 * np.pi / np.maximum(ell * (ell + 1), 1), 0.0)
    cls_ = np.stack([dl[k] * fac for k in ("TT", "EE", "BB", "TE")])
    if nfields == 2:
        cls_[0] = 0.0
        cls_[3] = 0.0
    np.random.seed(seed)
    maps = synfast(cls_, N, L, np.radians(0.5))
    g = torch.Generator(device="cuda").manual_seed(seed + 1)
    sig = torch.tensor([40.0, 0.2, 0.2], dtype=torch.float64, device="cuda")[:, None]
    d = maps + sig * torch.randn(maps.shape, dtype=torch.float64, device="cuda", generator=g)
    mask = band_mask(N) if mask_kind == "band" else galactic_mask(N)
    d = (d * torch.from_numpy(mask).cuda()).cpu().numpy()
    return d, mask, dl


def masked_c5_setup(args, ctx):
    """configs[4]'s per-iteration step (the closure run_masked times;
    tools/step_traffic.py counts its HBM bytes)."""
    import torch
    from gibbssampler_amd import _capi
    from gibbssampler_amd.engine import GibbsPlan
    from gibbssampler_amd.masked import MaskedCR
    from gibbssampler_amd.problem import gauss_beam
    L, N = args.lmax, args.nside
    NR = (L + 1) ** 2
    B = args.nchains
    d, mask, dl = _masked_data(N, L, 3)
    bl = gauss_beam(np.radians(0.5), L)
    cr = MaskedCR({"T": d[0], "Q": d[1], "U": d[2]}, 40.0 ** 2, 0.2 ** 2, bl, L, N, mask=mask, nfields=3,
                  gibbs_cr=True, n_gibbs=1, rng="native", seed=args.seed, chain=ctx.chain0, nchains=B)
    del d
    bins = {s: np.arange(0, L + 2) for s in ("TT", "EE", "BB", "TE")}
    plan = GibbsPlan(L, N, 3, B, bl, [1.0, 1.0, 1.0], bins, chain0=ctx.chain0)
    d0 = plan.zeros(1, 3, NR)
    dl1 = np.stack([dl[k] for k in ("TT", "EE", "BB", "TE")])
    dl_t = torch.from_numpy(np.array(np.broadcast_to(dl1, (B,) + dl1.shape))).cuda().contiguous()
    s = torch.zeros((B, 3, NR), dtype=torch.float64, device="cuda")
    it = [0]

    def step():
        it[0] += 1
        cr.step(_capi.GS_MCR_AUX, dl_t, s, iteration=it[0])
        st = plan.sweep_stats(d0, s)
        out = plan.cls_draw(st, None, seed=args.seed, iteration=it[0])
        dl_t.copy_(out[:, :, :L + 1])          # unbinned bins: bin b = l

    return step


def run_masked(args, ctx, cpu=None):
    """BASELINE configs[4]: CenteredGibbs TEB, masked (f_sky 0.8), aux-variable CR
    with n_gibbs = 1 (a9, TEB) + inverse-Wishart / inverse-Gamma C_l draw, one
    chain per GPU.  Per iteration: b s -> alm2map (TEB) -> v | s -> map2alm
    (TEB) -> s | v, then the sweep statistics and the C_l draw; all on the device."""
    import torch
    from gibbssampler_amd.sht import HealpixSHT
    L, N = args.lmax, args.nside
    Npix = 12 * N * N
    NR = (L + 1) ** 2
    B = args.nchains
    step = masked_c5_setup(args, ctx)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ctx.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    elapsed = ctx.max(time.perf_counter() - t0)
    # the transforms the step runs, timed with events on the launch stream
    sht = HealpixSHT(N, L)
    a = torch.zeros((3, NR), dtype=torch.float64, device="cuda")
    mp = torch.zeros((3, Npix), dtype=torch.float64, device="cuda")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    reps = 3
    ev[0].record()
    for _ in range(reps):
        sht.alm2map(a, ncomp=3, out=mp)
    ev[1].record()
    for _ in range(reps):
        sht.map2alm(mp, iter=0, ncomp=3, out=a)
    ev[2].record()
    torch.cuda.synchronize()
    t_syn = ev[0].elapsed_time(ev[1]) / reps
    t_ana = ev[1].elapsed_time(ev[2]) / reps
    if ctx.rank != 0:
        return None
    fl = sht_flops(N, L, 20)
    achieved = 2 * fl / ((t_syn + t_ana) * 1e-3) / 1e12
    # HBM bytes of one whole step (every kernel between two markers,
    # tools/step_traffic.py + tools/summarize_step_traffic.py): profiles/pmc_traffic.json
    tp = load_profile(args.profile_json, f"step_masked_N{N}_L{L}_B{B}_{args.mask}")
    return {
        "metric": METRIC % (N, L),
        "value": round(args.steps * B * ctx.world / elapsed, 4),
        "unit": "chain-iterations/s",
        "n_gpus": ctx.world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (analytic fiducial spectra, synfast on the device + white noise, 80% band mask)",
        "config": {"workload": "centered TEB masked aux-variable CR (n_gibbs=1)", "nside": N, "lmax": L,
                   "nfields": 3, "chains_per_gpu": B, "global_chains": B * ctx.world,
                   "rng": "native philox4x32-10", "parallelism": f"chains sharded over {ctx.world} GPU(s)"},
        "roofline": {"bound": "fp64", "kernel": "gs_sht alm2map + map2alm (TEB)", "achieved": round(achieved, 2),
                     "peak": FP64_VALU_PEAK_TFS, "unit": "TFLOP/s", "frac": round(achieved / FP64_VALU_PEAK_TFS, 4),
                     "traffic": tp.get("hbm_bytes_per_step"),
                     "traffic_unit": "HBM bytes per step (every kernel of one step, PMC)",
                     "traffic_over_algorithmic": tp.get("traffic_over_algorithmic"),
                     "algorithmic_bytes_per_step": tp.get("algorithmic_bytes_per_step"),
                     "traffic_source": tp.get("source"),
                     "algorithmic_flops_per_launch": fl,
                     "avg_launch_ms": {"alm2map": round(t_syn, 3), "map2alm": round(t_ana, 3)}},
        "cpu_baseline": _finalize_cpu(cpu),
        "notes": "healpy is absent: the CPU leg's transforms are oracle/sht_cpu.cpp (C++/OpenMP); see DESIGN.md",
    }


def masked_head_setup(args, ctx):
    """HEAD's masked run modes (run_masked_head's set-up, warm-up included):
    returns (runner, go, n_sht, what, pcg); go() runs the timed --steps
    iterations (tools/step_traffic.py counts their HBM bytes)."""
    import torch
    from gibbssampler_amd import gibbs as G
    from gibbssampler_amd.masked import MaskedRunner
    from gibbssampler_amd.problem import default_bins, default_blocks, proposal_variances, gauss_beam, bin_spectrum
    L, N = args.lmax, args.nside
    Npix = 12 * N * N
    B = args.nchains
    d, mask, dl = _masked_data(N, L, 2, mask_kind=args.mask)
    pix = {"Q": d[1], "U": d[2]}
    bins = default_bins(L, 2)
    blocks = default_blocks(L, bins)
    bl = gauss_beam(np.radians(0.5), L)
    pv = proposal_variances(L, N, bins, bl, 0.2 ** 2, 40.0 ** 2, fsky=float(np.mean(mask)))
    init = {s: bin_spectrum(dl[s], bins[s]) for s in ("EE", "BB")}
    noise_t, noise_p = np.ones(Npix) * 40.0 ** 2, np.ones(Npix) * 0.2 ** 2
    kw = dict(mask_path=mask, polarization=True, bins=bins, rng="native", seed=args.seed, chain0=ctx.chain0,
              nchains=B)
    pcg = None
    # the warm-up's last D_l of every chain (histories carry a chain axis for B > 1)
    last_of = lambda h: ({s: h[s][-1] for s in h} if B == 1 else
                         [{s: h[s][-1][b] for s in h} for b in range(B)])
    if args.workload in ("masked_centered_ula", "masked_centered_pcg"):
        ula = args.workload == "masked_centered_ula"
        smp = G.CenteredGibbs(pix, noise_t, noise_p, 0.5, N, L, Npix, n_iter=args.warmup, gibbs_cr=ula, ula=ula,
                              **kw)
        runner = MaskedRunner(smp.constrained_sampler, smp.bins)
        if ula:
            n_sht, what = 6, "aux-variable CR (n_gibbs 1) + MALA (CenteredGibbs.py:831-834), EB"
        else:
            n_sht, what = None, ("PCG CR every iteration (CenteredGibbs.py:448-491, pcg_accuracy 1e-5, per-l "
                                 "preconditioner, device-resident CG) + C_l draw, EB")
            pcg = smp.constrained_sampler
        h = runner.run(init, max(args.warmup, 1), None)[0]
        last = last_of(h)
        go = lambda: runner.run(last, args.steps, runner.s)
    elif args.workload == "masked_noncentered":
        smp = G.NonCenteredGibbs(pix, noise_t, noise_p, 0.5, N, L, Npix, pv, metropolis_blocks=blocks,
                                 n_iter=args.warmup, all_sph=True, **kw)
        runner = smp.masked_runner
        pcg = runner.cr
        n_sht, what = None, ("PCG CR every iteration (NonCenteredGibbs.py:178-196, device-resident CG), C^-1/2, "
                             f"pixel-domain MH over {runner.mh.K} blocks decided on the device (f2), EB")
        h = runner.run(init, max(args.warmup, 1))[0]
        last = last_of(h)
        go = lambda: runner.run(last, args.steps, s_init=runner.s)
    else:
        smp = G.ASIS(pix, noise_t, noise_p, 0.5, N, L, Npix, pv, metropolis_blocks=blocks, n_iter=args.warmup,
                     all_sph=False, gibbs_cr=True, n_gibbs=20, overrelaxation=True, **kw)
        runner = smp.masked_runner
        # the over-relaxed CR's transforms: v | s (1 synthesis) then per iteration
        # s | v, v | s, s | v -- 1 + 20 x 3 = 61 in the reference, whose s | v opening
        # iteration k > 0 re-transforms the map the previous one transformed (its v
        # has not changed): 42 distinct ones, the count charged here; + the f2
        # residual synthesis and the non-centring's (2)
        n_sht, what = 42 + 2, ("over-relaxed aux CR n_gibbs 20 (CenteredGibbs.py:733-825), pixel-domain MH "
                               f"over {runner.mh.K} blocks decided on the device (f2), EB")
        h = runner.run(init, max(args.warmup, 1))[0]
        last = last_of(h)
        go = lambda: runner.run(last, args.steps, s_init=runner.s)
    return runner, go, n_sht, what, pcg


def run_masked_head(args, ctx, cpu=None):
    """HEAD's real run modes (main_polarization.py:109-126,154) through the
    drop-in class surface, EB, one chain per GPU, N_side 256 / L 512 with the
    reference's Planck BB bins and 1 + 134 Metropolis blocks (config.py:45-55):

      masked_centered_ula  CenteredGibbs(mask, gibbs_cr=True, ula=True): per
                           iteration the aux-variable CR + MALA composition
                           (CenteredGibbs.py:831-834) and the C_l draw;
      masked_asis          ASIS(mask, all_sph=False, gibbs_cr=True, n_gibbs=20,
                           overrelaxation=True): over-relaxed aux CR (61 SHTs),
                           centred C_l draw, the pixel-domain MH sweep (f2,
                           decided on the device), re-centring.

    The reference's init CR (the PCG) runs in the warm-up; the timed region
    continues the chain for --steps iterations."""
    import torch
    L, N = args.lmax, args.nside
    B = args.nchains
    runner, go, n_sht, what, pcg = masked_head_setup(args, ctx)
    torch.cuda.synchronize()
    ctx.barrier()
    torch.cuda.synchronize()
    n_solves0 = len(pcg.pcg_iterations) if pcg is not None else 0
    t0 = time.perf_counter()
    go()
    torch.cuda.synchronize()
    elapsed = ctx.max(time.perf_counter() - t0)
    if ctx.rank != 0:
        return None
    pcg_info = None
    if pcg is not None:
        its = pcg.pcg_iterations[n_solves0:]
        launched = pcg.pcg_launched[n_solves0:]
        work = pcg.pcg_work[n_solves0:]
        syncs = pcg.pcg_syncs[n_solves0:]
        # per CG iteration one alm2map + one map2alm; the rhs adds map2alm iter 3 (7 transforms);
        # the algorithmic work counts each chain's own (converged) iterations
        n_sht = 2 * float(np.mean(its)) + 7
        pcg_info = {"solves": len(its), "cg_iterations_per_solve": round(float(np.mean(its)), 1),
                    "cg_iterations_launched_per_solve": round(float(np.mean(launched)), 1),
                    "cg_iterations_transformed_per_chain_and_solve": round(float(np.mean(work)) / B, 1),
                    "host_syncs_per_solve": round(float(np.mean(syncs)), 2),
                    "ms_per_cg_iteration_launched": round(elapsed / args.steps * 1e3 / max(float(np.mean(launched)),
                                                                                           1.0), 4),
                    "tolerance": pcg.pcg_accuracy, "residual_last": pcg.pcg_residual,
                    "note": "a batch's CG runs until its slowest chain converges (launched >= per-chain count); "
                            "from each host state read on only the unconverged chains are transformed "
                            "(transformed per chain ~ the per-chain count) and converged chains' update kernels "
                            "return at once"}
    fl = n_sht * sht_flops(N, L, 16) * B
    achieved = fl / (elapsed / args.steps) / 1e12
    # HBM bytes of one whole step (every kernel between two markers,
    # tools/step_traffic.py + tools/summarize_step_traffic.py): profiles/pmc_traffic.json
    tprof = load_profile(args.profile_json, f"step_{args.workload}_N{N}_L{L}_B{B}_{args.mask}")
    return {
        "metric": METRIC % (N, L),
        "value": round(args.steps * B * ctx.world / elapsed, 4),
        "unit": "chain-iterations/s",
        "n_gpus": ctx.world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (analytic fiducial EB spectra, synfast on the device + white noise, 80% "
                + ("band mask" if args.mask == "band" else "galactic-like mask with a wavy edge") + ")",
        "config": {"workload": f"{args.workload}: {what}", "surface": "gibbssampler_amd.gibbs (drop-in classes)",
                   "mask": args.mask, "ring_pair_classes": dict(zip(("no_weight", "varying", "constant"),
                                                                   runner.cr.ring_classes)),
                   "nside": N, "lmax": L, "nfields": 2, "chains_per_gpu": B, "global_chains": B * ctx.world,
                   "batching": "the GPU's chains as one batch: every transform one batched SHT over the B maps",
                   "bins": "config.py:45 Planck BB", "blocks": "config.py:51-55",
                   "rng": "native philox4x32-10", "parallelism": f"chains sharded over {ctx.world} GPU(s)"},
        "roofline": {"bound": "fp64", "kernel": f"{n_sht:.1f} spin-2 SHT-equivalents per chain-iteration",
                     "achieved": round(achieved, 3), "peak": FP64_VALU_PEAK_TFS, "unit": "TFLOP/s",
                     "frac": round(achieved / FP64_VALU_PEAK_TFS, 4), "traffic": tprof.get("hbm_bytes_per_step"),
                     "traffic_unit": "HBM bytes per step (every kernel of one step, PMC)",
                     "traffic_over_algorithmic": tprof.get("traffic_over_algorithmic"),
                     "algorithmic_bytes_per_step": tprof.get("algorithmic_bytes_per_step"),
                     "traffic_source": tprof.get("source"),
                     "algorithmic_flops_per_step": fl},
        "cpu_baseline": _finalize_cpu(cpu, pcg_info["cg_iterations_per_solve"] if pcg_info else None),
        "pcg": pcg_info,
        "notes": "healpy is absent: the CPU leg's transforms are oracle/sht_cpu.cpp (C++/OpenMP) (DESIGN.md 7)",
    }


if __name__ == "__main__":
    main()
