"""CPU baseline of the SHT-bound (masked) bench workloads (TEST / MEASUREMENT
INFRASTRUCTURE: only bench.py's cpu_baseline leg runs it, as a child process).

The reference's masked samplers restated by oracle/masked.py, with the
transforms by oracle/sht_cpu.cpp (C++/OpenMP HEALPix SHT, the stand-in for
healpy's libsharp, which is absent offline), on min(CPU affinity, 32) threads
(32 = one GPU's share of the 8-GPU node's 256 cores).  One chain, numpy's RNG (the draws'
source does not change the work).  The reference's per-call work structure is
kept: the pixel-domain MH scores every Metropolis block with a full synthesis
(NonCenteredGibbs.py:333-355, 401-445), the over-relaxation runs its 1 + 3 n_gibbs
transforms (CenteredGibbs.py:733-825), the PCG runs the qcinv "diag_cl" CG.

Workloads (bench.py's names):
  masked               configs[4]: TEB aux-variable CR n_gibbs 1 + C_l draw, N_side 2048
  masked_centered_ula  aux CR + MALA (CenteredGibbs.py:831-834) + C_l draw, EB
  masked_asis          over-relaxed aux CR n_gibbs 20, C_l draw, non-centring, pixel MH, re-centring
  masked_centered_pcg  PCG CR + C_l draw
  masked_noncentered   PCG CR, C^-1/2, pixel MH

A PCG solve is sampled: ``--cg-sample`` CG iterations are timed and the solve
is scaled to ``--cg-iters`` iterations (bench.py passes the count its own device
solves took: same operator, preconditioner and tolerance).  Prints one JSON line.
"""
import argparse
import json
import time

import numpy as np

from . import harmonic as H
from . import masked as MK
from . import sht as O
from . import sht_cpu as C


def _problem(nside, lmax, nfields, seed=0):
    rng = np.random.default_rng(seed)
    npix = 12 * nside * nside
    th, _ = O.pixel_angles(nside)
    mask = (np.abs(np.cos(th)) > 0.2).astype(np.float64)
    del th
    sig2 = np.array([40.0 ** 2, 0.2 ** 2, 0.2 ** 2])
    maps = rng.normal(size=(3, npix)) * np.sqrt(sig2)[:, None] * mask[None]
    if nfields == 2:
        maps[0] = 0.0
    inv = mask[None] / sig2[:, None]
    if nfields == 2:
        inv[0] = 0.0
    bl = H.gauss_beam(np.radians(0.5), lmax)
    mm = MK.MaskedModel(lmax, nside, nfields, bl, maps, inv, sht=C.Auto)
    ell = np.arange(lmax + 1.0)
    dl = {"TT": np.where(ell >= 2, 1000.0, 0.0), "EE": np.where(ell >= 2, 10.0 * (ell / 100.0) ** 0.5, 0.0),
          "BB": np.where(ell >= 2, 0.01, 0.0)}
    dl["TE"] = 0.5 * np.sqrt(dl["TT"] * dl["EE"])
    spectra = H.SPECTRA[nfields]
    dl_un = np.stack([dl[s] for s in spectra])
    bins = {s: np.arange(lmax + 2) for s in spectra}
    model = H.Model(lmax, nside, nfields, bl, [1.0] * nfields, bins, d_alm=np.zeros((nfields, (lmax + 1) ** 2)))
    return mm, model, dl_un


def _mh_model(mm, lmax, nside):
    """the EB pixel-MH problem with the reference's Planck BB bins / 1 + 134 blocks at L 512."""
    from gibbssampler_amd.problem import default_bins, default_blocks, proposal_variances
    bins = default_bins(lmax, 2)
    blocks = default_blocks(lmax, bins)
    pv = proposal_variances(lmax, nside, bins, mm.bl, 0.2 ** 2, 40.0 ** 2, fsky=0.8)
    return H.Model(lmax, nside, 2, mm.bl, [1.0, 1.0], bins, blocks=blocks, proposal_variances=pv,
                   d_alm=np.zeros((2, (lmax + 1) ** 2)))


def _cls_draw(model, s):
    """the centered C_l draw from the map's statistics (CenteredGibbs.py:54-93)"""
    return H.centered_cls_draw(model, H.sweep_stats(model, s, model.d_alm), seed=1, chain=0, iteration=1)


def _binned(mh, un):
    """bin means of unbinned D_l (dict spectrum -> [L+1]) on the MH model's bins"""
    return {sp: np.add.reduceat(un[sp], mh.bins[sp][:-1]) / np.diff(mh.bins[sp]) for sp in mh.spectra}


def _pcg_sampled(mm, dl_un, n_sample, tol):
    """the PCG CR with its solve cut at n_sample CG iterations: (seconds of the
    rhs, seconds per CG iteration, the map)."""
    draws = MK.ReplayDraws()
    t0 = time.perf_counter()
    z_pix = draws.pixel_normals(mm.F, mm.Npix)
    z_slot = draws.slot_normals(mm.F, (mm.L + 1) ** 2)
    rhs = mm.second_part_grad() + MK.pcg_fluctuation(mm, dl_un, z_pix, z_slot)
    t1 = time.perf_counter()
    x, it = MK.pcg_solve(mm, dl_un, rhs, tol=tol, maxiter=n_sample)
    t2 = time.perf_counter()
    return t1 - t0, (t2 - t1) / max(it, 1), x


def run(workload, nside, lmax, cg_iters=None, cg_sample=10):
    threads = C.threads()
    nfields = 3 if workload == "masked" else 2
    t_build = time.perf_counter()
    mm, model, dl_un = _problem(nside, lmax, nfields)
    mm.second_part_grad()
    C.build()
    setup = time.perf_counter() - t_build
    rng = np.random.default_rng(3)
    s = rng.normal(size=(nfields, (lmax + 1) ** 2)) * 1e-3
    np.random.seed(11)
    draws = MK.ReplayDraws()
    parts = None
    t0 = time.perf_counter()
    if workload == "masked":
        s, _ = MK.aux_variable(mm, dl_un, s, 1, draws)
        _cls_draw(model, s)
        sample = "one full iteration: TEB aux-variable CR (n_gibbs 1) + inverse-Wishart / inverse-Gamma C_l draw"
        per_it = time.perf_counter() - t0
    elif workload == "masked_centered_ula":
        s, _ = MK.sample_dispatch(mm, dl_un, s, draws, gibbs_cr=True, overrelaxation_flag=False, ula=True,
                                  n_gibbs=1, noise_pol0=0.2 ** 2)
        _cls_draw(model, s)
        sample = "one full iteration: aux-variable CR + MALA + C_l draw, EB"
        per_it = time.perf_counter() - t0
    elif workload == "masked_asis":
        mh = _mh_model(mm, lmax, nside)
        s, _ = MK.sample_dispatch(mm, dl_un, s, draws, gibbs_cr=True, overrelaxation_flag=True, ula=False,
                                  n_gibbs=20, noise_pol0=0.2 ** 2)
        start = _binned(mh, _cls_draw(model, s))
        s_nc = MK.noncentre(mm, mh.unfold(start), s)
        new, _ = MK.pixel_mh(mm, mh, start, s_nc, seed=5, chain=0, iteration=1)
        MK.noncentre(mm, mh.unfold(new), s, inverse=False)
        sample = (f"one full iteration: over-relaxed aux CR n_gibbs 20 (61 transforms), C_l draw, non-centring, "
                  f"pixel-domain MH over {sum(len(b) - 1 for b in mh.blocks.values())} blocks, one full synthesis "
                  f"per block (NonCenteredGibbs.py:333-355), re-centring, EB")
        per_it = time.perf_counter() - t0
    elif workload in ("masked_centered_pcg", "masked_noncentered"):
        t_rhs, t_cg, x = _pcg_sampled(mm, dl_un, cg_sample, 1e-5)
        n_cg = cg_iters if cg_iters else cg_sample
        t_rest0 = time.perf_counter()
        if workload == "masked_centered_pcg":
            _cls_draw(model, x)
            what = "C_l draw"
        else:
            mh = _mh_model(mm, lmax, nside)
            start = _binned(mh, {sp: dl_un[k] for k, sp in enumerate(mh.spectra)})
            MK.pixel_mh(mm, mh, start, MK.noncentre(mm, dl_un, x), seed=5, chain=0, iteration=1)
            what = "C^-1/2 + pixel-domain MH (one full synthesis per block)"
        t_rest = time.perf_counter() - t_rest0
        per_it = t_rhs + n_cg * t_cg + t_rest
        sample = (f"PCG rhs ({t_rhs:.2f} s) + {{n_cg}} CG iterations at {t_cg:.3f} s each (timed: {cg_sample}; "
                  f"the count is the device solve's: same operator, per-l preconditioner, tolerance 1e-5) "
                  f"+ {what} ({t_rest:.2f} s), EB")
        parts = {"t_rhs": t_rhs, "t_cg": t_cg, "t_rest": t_rest, "n_sampled": cg_sample}
    else:
        raise ValueError(workload)
    wall = time.perf_counter() - t0
    return {"value": 1.0 / per_it, "unit": "chain-iterations/s", "cores": threads, "kind": "port",
            "sample": f"{sample}; N_side {nside}, l_max {lmax}; transforms by oracle/sht_cpu.cpp (C++/OpenMP, "
                      f"{threads} threads); {wall:.1f} s timed (setup {setup:.1f} s untimed)",
            "seconds_per_iteration": per_it, "pcg_parts": parts}


def finalize(r, cg_iters=None):
    """the baseline line for bench.py: a PCG workload's rate with the device
    solve's CG iteration count (``{n_cg}`` in the sample text)."""
    if r is None:
        return None
    out = {k: r[k] for k in ("value", "unit", "cores", "kind", "sample")}
    p = r.get("pcg_parts")
    if p:
        # the CPU leg times p["n_sampled"] CG iterations and extrapolates to a whole
        # solve: with the device solve's iteration count when given, else the
        # sampled count itself (the CPU PCG is never run to convergence)
        n = float(cg_iters) if cg_iters is not None else float(p.get("n_sampled", 0) or 0)
        if n <= 0:
            return None
        out["value"] = 1.0 / (p["t_rhs"] + n * p["t_cg"] + p["t_rest"])
        out["sample"] = r["sample"].replace("{n_cg}", f"{n:.1f}")
        out["extrapolated"] = (f"per-CG-iteration time measured over {p.get('n_sampled', '?')} CG iterations, "
                               f"times {n:.1f} iterations per solve"
                               + (" (the GPU solve's count)" if cg_iters is not None else " (the sampled count)"))
    out["value"] = round(out["value"], 6)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", required=True)
    ap.add_argument("--nside", type=int, required=True)
    ap.add_argument("--lmax", type=int, required=True)
    ap.add_argument("--cg-iters", type=int, default=None)
    ap.add_argument("--cg-sample", type=int, default=10)
    a = ap.parse_args()
    import sys
    import threading
    t0 = time.time()

    def beat():                      # a progress line every 30 s (long runs stay visibly alive)
        while True:
            time.sleep(30)
            print(f"cpu baseline {a.workload}: {time.time() - t0:.0f} s", file=sys.stderr, flush=True)

    threading.Thread(target=beat, daemon=True).start()
    print(json.dumps(run(a.workload, a.nside, a.lmax, a.cg_iters, a.cg_sample)))


if __name__ == "__main__":
    main()
