"""Cost split of the NC prologue's three roles at configs[2] (32 TEB chains,
L 1024): the MH proposals (gs_mh_propose with uniforms), the CR block
parameters (gs_block_params) and the whole fused prologue (gs_nc_prologue),
each timed over many launches with events on the launch stream.

usage (GPU box): python tools/prologue_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gibbssampler_amd import _capi as C  # noqa: E402
from gibbssampler_amd.problem import synthetic_problem  # noqa: E402
from gibbssampler_amd.samplers import BatchedRunner  # noqa: E402


def timed(fn, n=200):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def main():
    P = synthetic_problem(1024, 512, 3, seed=0)
    r = BatchedRunner("noncentered", P["lmax"], P["nside"], 3, 32, P["bl"], P["noise_var"], P["bins"], P["d_alm"],
                      blocks=P["blocks"], proposal_variances=P["proposal_variances"], rng="native", seed=5,
                      store_skymap=False)
    r.init(P["dls_init"])
    p = r.plan
    prop = p.zeros(p.nchains, p.nspec, p.maxbins)
    logr = p.zeros(p.nchains, p.nspec, p.maxbins)
    ua = p.zeros(p.nchains, max(p.nacc, 1))
    params = p.zeros(p.nchains, p.L + 1, C.GS_NPARAM)
    s = p._s()
    t_prop = timed(lambda: C.check(p.lib.gs_mh_propose(p._h, C.ptr(r.dl), None, 5, 7, C.ptr(prop), C.ptr(logr),
                                                       C.ptr(ua), s)))
    t_par = timed(lambda: C.check(p.lib.gs_block_params(p._h, C.GS_MODE_NONCENTERED, C.ptr(r.dl), C.ptr(params), s)))
    t_pro = timed(lambda: p.nc_prologue(r.dl, seed=5, iteration=7))
    print(f"proposals + uniforms (2 launches + 2 memsets): {t_prop:7.2f} us")
    print(f"block parameters (1 launch):                 {t_par:7.2f} us")
    print(f"fused prologue (1 launch):                   {t_pro:7.2f} us")


if __name__ == "__main__":
    main()
