"""Chain lanes: the chains of one GPU split into G independent groups, each a
BatchedRunner with its own K-step hipGraph, the G graphs replayed on G streams
at once -- so one group's step tail (statistics finish, MH decisions, prologue:
a few dozen workgroups) runs beside another group's CR sweep instead of on an
otherwise idle chip.  Compared in ONE process against the single-graph run of
all chains, interleaved; and checked bit for bit (chain c of a lane = chain c
of the one-group run: the plans are chain-count independent).

usage (GPU box):  python tools/lanes_probe.py [KIND L NSIDE NCHAINS STEPS G1 G2 ...]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gibbssampler_amd.problem import synthetic_problem  # noqa: E402
from gibbssampler_amd.samplers import BatchedRunner  # noqa: E402


def make(P, kind, nch, c0, steps):
    r = BatchedRunner(kind, P["lmax"], P["nside"], 3, nch, P["bl"], P["noise_var"], P["bins"], P["d_alm"],
                      blocks=P["blocks"], proposal_variances=P["proposal_variances"], rng="native", seed=5,
                      chain0=c0, store_skymap=False)
    r.init(P["dls_init"])
    r.capture_steps(steps)
    return r


def capture_branches(rs, steps):
    """ONE hipGraph holding every lane's K steps as its own branch (forked from
    the capture stream once, joined once at the end); noncentered only."""
    from gibbssampler_amd.samplers import _capture
    for r in rs:
        r.plan.iteration_counter(True, r.iteration + 1)
    torch.cuda.synchronize()
    sts = [torch.cuda.Stream() for _ in rs]
    g = torch.cuda.CUDAGraph()
    with _capture(g):
        cap = torch.cuda.current_stream()
        for s in sts:
            s.wait_stream(cap)
        for i in range(steps):
            for r, s in zip(rs, sts):
                p = r.plan
                with torch.cuda.stream(s):
                    p.graph_step(i, steps if i == steps - 1 else 0)
                    p.nc_prologue(r.dl, seed=r.seed)
                    p.nc_sweep(r.d, r.dl, r.s, seed=r.seed, finish=False)
                    p.nc_finish()
                    p.nc_decide_fused(r.dl, seed=r.seed, accept=r.accept)
        for s in sts:
            cap.wait_stream(s)
    for r in rs:
        r.plan.graph_step(0, 1)
    return g


class Branched:
    def __init__(self, rs, steps):
        self.rs, self.steps = rs, steps
        self.g = capture_branches(rs, steps)

    def step(self):
        self.g.replay()
        for r in self.rs:
            r.iteration += self.steps


def main(kind="noncentered", L=1024, nside=512, nch=32, steps=200, *groups, rounds=7):
    L, nside, nch, steps = int(L), int(nside), int(nch), int(steps)
    groups = [g for g in groups] or ["1", "2", "4"]
    # "G@C": G lanes, lane g's replay started behind a spin of g * C clock
    # cycles (torch.cuda._sleep) -- lanes out of phase, one's tail beside another's sweep
    offs = {g: int(g.split("@")[1]) if "@" in g else 0 for g in groups}
    groups_n = {g: int(g.split("@")[0].rstrip("g")) for g in groups}
    P = synthetic_problem(L, nside, 3, seed=0)
    setups = {}
    built = {}
    for G in groups:
        n = groups_n[G]
        if G.endswith("g"):
            # "Gg": G lanes as branches of one graph
            n = int(G[:-1])
            per = nch // n
            rs = [make(P, kind, per, g * per, 1) for g in range(n)]
            setups[G] = ([Branched(rs, steps)], [torch.cuda.Stream()])
            continue
        if n not in built:
            per = nch // n
            built[n] = ([make(P, kind, per, g * per, steps) for g in range(n)], [torch.cuda.Stream() for _ in range(n)])
        setups[G] = built[n]
    res = {G: [] for G in groups}
    for rnd in range(rounds):
        for G, (rs, sts) in setups.items():
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for j, (r, s) in enumerate(zip(rs, sts)):
                s.wait_event(e0)
                with torch.cuda.stream(s):
                    if j and offs[G]:
                        torch.cuda._sleep(j * offs[G])
                    r.step()
            for s in sts:
                torch.cuda.current_stream().wait_stream(s)
            e1.record()
            torch.cuda.synchronize()
            if rnd:
                res[G].append(e0.elapsed_time(e1) / steps)
    for G in groups:
        print(f"lanes {G}: {np.median(res[G]) * 1e3:8.2f} us/step (min {min(res[G]) * 1e3:8.2f})", flush=True)
    # bit-identity: every lane's D_l against the one-group run (same number of steps)
    def dls(G):
        rs = setups[G][0]
        rs = rs[0].rs if isinstance(rs[0], Branched) else rs
        return torch.cat([r.dl for r in rs], 0)
    ref = dls(groups[0])
    for G in groups[1:]:
        if offs[G]:
            continue
        got = dls(G)
        print(f"lanes {G} == lanes {groups[0]}: {bool(torch.equal(got, ref))}", flush=True)

    # the same lanes one after another on one stream (each lane's own step time)
    for G, (rs, _) in setups.items():
        if offs[G] or G.endswith("g"):
            continue
        t = []
        for rnd in range(3):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for r in rs:
                r.step()
            e1.record()
            torch.cuda.synchronize()
            t.append(e0.elapsed_time(e1) / steps)
        print(f"lanes {G} serial: {np.median(t) * 1e3:8.2f} us/step", flush=True)

if __name__ == "__main__":
    main(*sys.argv[1:])
