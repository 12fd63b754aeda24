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
    ap.add_argument("--workload", default="noncentered", choices=["noncentered", "centered", "asis", "masked"],
                    help="masked = BASELINE configs[4]: CenteredGibbs TEB with an 80%% mask, aux-variable CR "
                         "(n_gibbs 1), N_side 2048 / l_max 4096, 1 chain per GPU")
    ap.add_argument("--nchains", type=int, default=None, help="chains per GPU (32; masked: 1)")
    ap.add_argument("--lmax", type=int, default=None, help="1024 (masked: 4096)")
    ap.add_argument("--nside", type=int, default=None, help="512 (masked: 2048)")
    ap.add_argument("--fields", type=int, default=3, choices=[1, 2, 3])
    ap.add_argument("--seed", type=int, default=20261015)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of one hipGraph of the timed steps")
    ap.add_argument("--time-every", type=int, default=1,
                    help="bracket the CR sweep of every N-th timed step with hipEvents (graph mode)")
    ap.add_argument("--profile-json", default=os.path.join(HERE, "profiles", "pmc_traffic.json"))
    a = ap.parse_args()
    masked = a.workload == "masked"
    a.nchains = a.nchains or (1 if masked else 32)
    a.lmax = a.lmax or (4096 if masked else 1024)
    a.nside = a.nside or (2048 if masked else 512)
    return a


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
    if args.workload == "masked":
        return run_masked(args, rank, world, dist)
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
    one_graph = not args.no_graph
    if one_graph:
        # the K timed iterations as ONE hipGraph (D_l trace written on the device);
        # every CR-sweep kernel is bracketed by event-record nodes inside the graph,
        # so its duration is measured on its stream over the timed region itself
        # (--time-every N brackets only every N-th sweep: an event node costs ~5 us)
        runner.capture_steps(args.steps, trace=traces[0], trace_capacity=args.steps, time_sweeps=True,
                             time_every=args.time_every)
    else:
        for p in plans:
            p.sweep_timing(True)        # events around every sweep launch of the timed loop
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if one_graph:
        runner.step()                   # one replay = the K steps
    else:
        for i in range(args.steps):
            runner.step()
            traces[0][i].copy_(runner.dl)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if dist is not None:
        dist.barrier()
    elapsed = t1 - t0
    timed = [p.sweep_timing(False) for p in plans]
    timing_mode = ("hipEvents around each sweep inside the timed graph" if one_graph else
                   "hipEvents around each sweep of the timed loop")
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
                       "launch": "one hipGraph of all timed iterations" if one_graph else "eager",
                       "nside": args.nside, "lmax": args.lmax, "nfields": args.fields,
                       "chains_per_gpu": args.nchains, "global_chains": args.nchains * world,
                       "rng": "native philox4x32-10", "parallelism": f"chains sharded over {world} GPU(s)"},
            "roofline": {"bound": "hbm", "kernel": "k_cr_sweep", "achieved": round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "algorithmic_bytes_per_launch": alg_bytes,
                         "avg_launch_ms": round(sweep_avg_ms, 5), "launches": sweep_n, "timing": timing_mode},
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


FP64_VALU_PEAK_TFS = 78.6   # MI355X_MICROARCH.md: FP64 vector


def sht_flops(nside, L, ncomp_c=20):
    """N_ringpair * N_lm * c (c = 4 spin-0 + 16 spin-2 = 20 for TEB)."""
    return 2 * nside * (L + 1) * (L + 2) // 2 * ncomp_c


def run_masked(args, rank, world, dist):
    """BASELINE configs[4]: CenteredGibbs TEB, masked (f_sky 0.8), aux-variable CR
    with n_gibbs = 1 (a9, TEB) + inverse-Wishart / inverse-Gamma C_l draw, one
    chain per GPU.  Per iteration: b s -> alm2map (TEB) -> v | s -> map2alm
    (TEB) -> s | v, then the sweep statistics and the C_l draw; all on the device."""
    from gibbssampler_amd import _capi
    from gibbssampler_amd.data import band_mask, synfast
    from gibbssampler_amd.engine import GibbsPlan
    from gibbssampler_amd.masked import MaskedCR
    from gibbssampler_amd.problem import fiducial_dl, gauss_beam
    from gibbssampler_amd.sht import HealpixSHT
    L, N = args.lmax, args.nside
    Npix = 12 * N * N
    NR = (L + 1) ** 2
    if args.nchains != 1:
        raise SystemExit("masked workload: one chain per GPU (chains shard over GPUs)")
    dl = fiducial_dl(L, 3)
    ell = np.arange(L + 1, dtype=np.float64)
    fac = np.where(ell > 0, 2 * np.pi / np.maximum(ell * (ell + 1), 1), 0.0)
    cls_ = np.stack([dl[k] * fac for k in ("TT", "EE", "BB", "TE")])
    np.random.seed(0)
    fwhm = np.radians(0.5)
    maps = synfast(cls_, N, L, fwhm)                                   # [3, Npix] device
    g = torch.Generator(device="cuda").manual_seed(1)
    sig = torch.tensor([40.0, 0.2, 0.2], dtype=torch.float64, device="cuda")[:, None]
    d = maps + sig * torch.randn(maps.shape, dtype=torch.float64, device="cuda", generator=g)
    mask = band_mask(N)
    mt = torch.from_numpy(mask).cuda()
    d = (d * mt).cpu().numpy()
    del maps
    bl = gauss_beam(fwhm, L)
    cr = MaskedCR({"T": d[0], "Q": d[1], "U": d[2]}, 40.0 ** 2, 0.2 ** 2, bl, L, N, mask=mask, nfields=3,
                  gibbs_cr=True, n_gibbs=1, rng="native", seed=args.seed, chain=rank)
    del d
    bins = {s: np.arange(0, L + 2) for s in ("TT", "EE", "BB", "TE")}
    plan = GibbsPlan(L, N, 3, 1, bl, [1.0, 1.0, 1.0], bins, chain0=rank)
    d0 = plan.zeros(1, 3, NR)
    dl_t = torch.from_numpy(np.stack([dl[k] for k in ("TT", "EE", "BB", "TE")])).cuda().contiguous()
    s = torch.zeros((3, NR), dtype=torch.float64, device="cuda")
    it = [0]

    def step():
        it[0] += 1
        cr.step(_capi.GS_MCR_AUX, dl_t, s, iteration=it[0])
        st = plan.sweep_stats(d0, s[None])
        out = plan.cls_draw(st, None, seed=args.seed, iteration=it[0])
        dl_t.copy_(out[0, :, :L + 1])          # unbinned bins: bin b = l

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
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
    if rank == 0:
        fl = sht_flops(N, L)
        achieved = 2 * fl / ((t_syn + t_ana) * 1e-3) / 1e12
        line = {
            "metric": "Gibbs iters/sec (constrained-realization + C_l draw), Nside=%d lmax=%d" % (N, L),
            "value": round(args.steps * world / elapsed, 4),
            "unit": "chain-iterations/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (analytic fiducial spectra, synfast on the device + white noise, 80% band mask)",
            "config": {"workload": "centered TEB masked aux-variable CR (n_gibbs=1)", "nside": N, "lmax": L,
                       "nfields": 3, "chains_per_gpu": 1, "global_chains": world,
                       "rng": "native philox4x32-10", "parallelism": f"chains sharded over {world} GPU(s)"},
            "roofline": {"bound": "fp64", "kernel": "gs_sht alm2map + map2alm (TEB)", "achieved": round(achieved, 2),
                         "peak": FP64_VALU_PEAK_TFS, "unit": "TFLOP/s", "frac": round(achieved / FP64_VALU_PEAK_TFS, 4),
                         "traffic": None, "algorithmic_flops_per_launch": fl,
                         "avg_launch_ms": {"alm2map": round(t_syn, 3), "map2alm": round(t_ana, 3)}},
            "cpu_baseline": None,
            "notes": "healpy is absent, so no CPU SHT baseline at this size; see DESIGN.md",
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
