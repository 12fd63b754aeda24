#!/usr/bin/env python
"""Gibbs iterations/sec on MI355X -- BASELINE.json metric.

Workload (default, BASELINE.json configs[2]): NonCenteredGibbs TEB, all_sph
full sky, N_side = 512, l_max = 1024, 32 chains per GPU, synthetic data
(SURVEY.md 8d fiducial), native Philox RNG.  One "step" = one Gibbs
iteration (constrained realisation + C_l draw) of every chain on every GPU.

  python bench.py [--gpus N --steps K --warmup W --workload noncentered|centered|asis]

For N > 1 launch with torch.distributed.run (one rank per GPU, RCCL): chains
are sharded (global chain id = rank * chains_per_gpu + c), no collective runs
inside an iteration; the D_l traces are all-gathered once after the timed
region.  value = total chain-iterations / max-over-ranks wall time.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="noncentered", choices=["noncentered", "centered", "asis"])
    ap.add_argument("--nchains", type=int, default=32, help="chains per GPU")
    ap.add_argument("--lmax", type=int, default=1024)
    ap.add_argument("--nside", type=int, default=512)
    ap.add_argument("--fields", type=int, default=3, choices=[1, 2, 3])
    ap.add_argument("--seed", type=int, default=20261015)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of one hipGraph per step")
    ap.add_argument("--timing-launches", type=int, default=20,
                    help="eager steps after the timed loop whose sweep launches are timed with hipEvents")
    ap.add_argument("--profile-json", default=os.path.join(HERE, "profiles", "pmc_traffic.json"))
    return ap.parse_args()


def sweep_algorithmic_bytes(L, F, nchains, ntask_stats):
    """Unique HBM bytes one CR-sweep launch must move (DESIGN.md 'Roofline'):
    write s (8 F (L+1)^2 per chain) + read the shared data once (8 F (L+1)^2)
    + read the per-l operator table (80 B per chain and l) + write the per-task
    partial statistics."""
    NR = (L + 1) ** 2
    return 8 * F * NR * nchains + 8 * F * NR + 80 * (L + 1) * nchains + ntask_stats


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        print(f"warning: WORLD_SIZE={world} != --gpus {args.gpus}", file=sys.stderr)
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from gibbssampler_amd.build import build
    if rank == 0 or world == 1:
        build()
    if dist is not None:
        dist.barrier()
    from gibbssampler_amd.problem import synthetic_problem
    from gibbssampler_amd.samplers import BatchedRunner

    P = synthetic_problem(args.lmax, args.nside, args.fields, seed=0)
    runner = BatchedRunner(kind=args.workload, lmax=P["lmax"], nside=P["nside"], nfields=P["nfields"],
                           nchains=args.nchains, bl=P["bl"], noise_var=P["noise_var"], bins=P["bins"],
                           d_alm=P["d_alm"], blocks=P["blocks"], proposal_variances=P["proposal_variances"],
                           rng="native", seed=args.seed, chain0=rank * args.nchains)
    plans = (runner.plan,)
    runner.init(P["dls_init"])
    traces = [p.zeros(args.steps, p.nchains, p.nspec, p.maxbins) for p in plans]
    for _ in range(args.warmup):
        runner.step()
    use_graph = not args.no_graph
    if use_graph:
        # one hipGraph per Gibbs iteration: the D_l trace is written on the device
        runner.capture_graph(trace=traces[0], trace_capacity=args.steps)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        runner.step()
        if not use_graph:
            traces[0][i].copy_(runner.dl)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if dist is not None:
        dist.barrier()
    elapsed = t1 - t0
    # dominant-kernel timing: hipEvents around every sweep launch (on its stream) of
    # eager steps of the same state right after the timed loop
    runner.graph = None
    plans[0].iteration_counter(False)
    for p in plans:
        p.sweep_timing(True)
    for _ in range(args.timing_launches):
        runner.step()
    torch.cuda.synchronize()
    timed = [p.sweep_timing(False) for p in plans]
    trace = torch.cat(traces, 1)
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        # the run's only collective: gather every rank's D_l traces (RCCL over xGMI)
        gathered = [torch.empty_like(trace) for _ in range(world)]
        dist.all_gather(gathered, trace)
        torch.cuda.synchronize()
    total_chain_iters = args.steps * args.nchains * world
    value = total_chain_iters / elapsed
    ms_per_step = elapsed / args.steps * 1e3

    if rank == 0:
        sweep_n = sum(n for _, n in timed)
        sweep_ms = sum(ms for ms, _ in timed)
        sweep_avg_ms = sweep_ms / max(sweep_n, 1)
        per_launch = [sweep_algorithmic_bytes(p.L, p.F, p.nchains, p.nchains * p.ntask * p.nstat * 64 * 8)
                      for p in plans]
        alg_bytes = int(round(sum(b * n for b, (_, n) in zip(per_launch, timed)) / max(sweep_n, 1)))
        achieved = alg_bytes / (sweep_avg_ms * 1e-3) / 1e9
        plan = plans[0]
        traffic = None
        try:
            with open(args.profile_json) as f:
                prof = json.load(f)
            key = f"{args.workload}_L{args.lmax}_F{args.fields}_c{plan.nchains}"
            if key in prof:
                traffic = prof[key].get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            pass
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(P, args)
        line = {
            "metric": "Gibbs iters/sec (constrained-realization + C_l draw), Nside=512 lmax=1024",
            "value": round(value, 3),
            "unit": "chain-iterations/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (analytic fiducial spectra, d = b s + n in harmonic space, seed 0)",
            "config": {"workload": f"{args.workload} TEB all_sph full-sky" if args.fields == 3 else args.workload,
                       "launch": "hipGraph per iteration" if use_graph else "eager",
                       "nside": args.nside, "lmax": args.lmax, "nfields": args.fields,
                       "chains_per_gpu": args.nchains, "global_chains": args.nchains * world,
                       "rng": "native philox4x32-10", "parallelism": f"chains sharded over {world} GPU(s)"},
            "roofline": {"bound": "hbm", "kernel": "k_cr_sweep", "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "algorithmic_bytes_per_launch": alg_bytes,
                         "avg_launch_ms": round(sweep_avg_ms, 5), "launches": sweep_n},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def cpu_baseline(P, args):
    """Bounded sample of the same workload on one host core (oracle port)."""
    from oracle import harmonic as H
    from oracle.cpu_baseline import time_noncentered
    m = H.Model(P["lmax"], P["nside"], P["nfields"], P["bl"], P["noise_var"], P["bins"], P["blocks"],
                P["proposal_variances"], P["d_alm"])
    rate, n, dt = time_noncentered(m, P["dls_init"], budget_s=args.cpu_budget, max_iter=3)
    return {"value": round(rate, 5), "unit": "chain-iterations/s", "cores": 1, "kind": "port",
            "sample": f"{n} NonCentered TEB all_sph iteration(s) of 1 chain at Nside={P['nside']} "
                      f"lmax={P['lmax']} in {dt:.1f} s (vectorised numpy port with the reference's "
                      f"per-block full-sky likelihood, oracle/cpu_baseline.py)"}


if __name__ == "__main__":
    main()
