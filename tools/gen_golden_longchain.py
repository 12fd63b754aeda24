"""Long-chain oracle fixture for the headline configuration.

BASELINE configs[2]: NonCenteredGibbs TEB all_sph, N_side 512, l_max 1024, the
synthetic problem of bench.py (gibbssampler_amd.problem.synthetic_problem, seed
0), native Philox streams, seed 20261015.  The oracle (oracle/harmonic.py:
cr_normals -> cr_apply -> sweep_stats -> nc_mh, NonCenteredGibbs.py:134-176,
401-445, 546-560) runs chains 0..3 for NITER iterations from the same start
D_l; the fixture keeps, per chain / spectrum / bin, the mean of the binned D_l
over the iterations (the north_star's "sampled C_l means"), the D_l after
iterations 1, NITER/2 and NITER, and the accept counts.  The GPU test
(tests/test_gpu_longchain.py) runs the same chains through BatchedRunner and
compares: means within 1e-6 relative, the north_star bar.

usage: python tools/gen_golden_longchain.py [--niter 100] [--procs 4]
-> tests/golden/longchain_nc_teb_L1024_c4.npz  (~9 min on 4 cores)
"""
import argparse
import multiprocessing as mp
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SEED = 20261015
OUT = os.path.join(ROOT, "tests", "golden", "longchain_nc_teb_L1024_c4.npz")
SPECTRA = ("TT", "EE", "BB", "TE")


def run_chain(args):
    chain, niter = args
    from gibbssampler_amd.problem import synthetic_problem
    from oracle import harmonic as H
    P = synthetic_problem(1024, 512, 3, seed=0)
    m = H.Model(P["lmax"], P["nside"], 3, P["bl"], P["noise_var"], P["bins"], P["blocks"],
                P["proposal_variances"], P["d_alm"])
    dl = {k: np.array(v, dtype=np.float64) for k, v in P["dls_init"].items()}
    nb = {sp: len(P["bins"][sp]) - 1 for sp in SPECTRA}
    acc_sum = {sp: 0 for sp in SPECTRA}
    total = {sp: np.zeros(nb[sp]) for sp in SPECTRA}
    snaps = {}
    t0 = time.time()
    for it in range(1, niter + 1):
        M, Lc = H.noncentered_params(m, m.unfold(dl))
        z = np.stack([H.cr_normals(SEED, chain, it, 0, f, m.L) for f in range(3)])
        s = H.cr_apply(m, M, Lc, m.d_alm, z)
        st = H.sweep_stats(m, s, m.d_alm)
        del s, z
        dl, acc = H.nc_mh(m, dl, st, seed=SEED, chain=chain, iteration=it)
        for sp in SPECTRA:
            total[sp] += np.asarray(dl[sp])[:nb[sp]]
            acc_sum[sp] += int(np.sum(acc[sp]))
        if it in (1, niter // 2, niter):
            snaps[it] = {sp: np.asarray(dl[sp])[:nb[sp]].copy() for sp in SPECTRA}
        if it % 10 == 0:
            print(f"chain {chain}: iteration {it} ({time.time() - t0:.0f} s)", flush=True)
    return chain, {sp: total[sp] / niter for sp in SPECTRA}, snaps, acc_sum


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--niter", type=int, default=100)
    ap.add_argument("--procs", type=int, default=4)
    ap.add_argument("--chains", type=int, default=4)
    a = ap.parse_args()
    with mp.get_context("spawn").Pool(a.procs) as pool:
        res = sorted(pool.map(run_chain, [(c, a.niter) for c in range(a.chains)]), key=lambda r: r[0])
    out = {"seed": np.int64(SEED), "niter": np.int64(a.niter), "nchains": np.int64(a.chains),
           "config": np.array("noncentered TEB all_sph, N_side 512, l_max 1024, synthetic_problem(seed=0)")}
    snap_its = sorted(res[0][2])
    out["snapshot_iterations"] = np.array(snap_its, dtype=np.int64)
    for sp in SPECTRA:
        out[f"mean_{sp}"] = np.stack([r[1][sp] for r in res])
        out[f"accepts_{sp}"] = np.array([r[3][sp] for r in res], dtype=np.int64)
        out[f"snap_{sp}"] = np.stack([np.stack([r[2][it][sp] for it in snap_its]) for r in res])
    np.savez_compressed(OUT, **out)
    print(f"wrote {OUT}")


if __name__ == "__main__":
    main()
