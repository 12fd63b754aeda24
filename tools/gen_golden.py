"""Generate golden vectors by running the REFERENCE's own Python (build container only).

Usage:  python tools/gen_golden.py [--ref /root/reference] [--out tests/golden]

The reference (Gabriel-Ducrocq/GibbsSampler) imports healpy, qcinv and classy,
none of which exist offline.  This script writes throw-away stand-ins for
those three third-party packages into a temporary directory (never into the
repo) and then imports the reference modules unchanged:

  * healpy: gauss_beam / alm2cl / npix2nside / nside2resol restated from their
    published definitions; read_map / ud_grade return an all-ones mask;
    map2alm / alm2map return zeros -- they are only touched by constructors
    (CenteredGibbs.py:298 second_part_grad) whose output no fixture depends on.
  * qcinv: inert objects for the constructors (ConstrainedRealization.py:40-41,
    CenteredGibbs.py:281-282).  The PCG branch itself is never executed: the
    full-sky Centered/ASIS drivers are run with the CR dispatcher routed to the
    closed-form ``sample_no_mask`` (CenteredGibbs.py:317), its exact limit.
  * classy: an empty Class (utils.py:7).

Only inputs and outputs (numbers) are written to tests/golden/*.npz, together
with the numpy / scipy versions.  No reference source enters the repo.
"""
import argparse
import contextlib
import io
import os
import sys
import tempfile
import time
import types

import numpy as np
import scipy

HEALPY_STUB = '''
import numpy as np
def gauss_beam(fwhm, lmax=512, pol=False):
    sigma = fwhm / np.sqrt(8.0 * np.log(2.0))
    ell = np.arange(lmax + 1)
    return np.exp(-0.5 * ell * (ell + 1) * sigma ** 2)
def npix2nside(npix):
    return int(round(np.sqrt(npix / 12)))
def nside2npix(nside):
    return 12 * nside * nside
def nside2resol(nside, arcmin=False):
    r = np.sqrt(4 * np.pi / (12 * nside * nside))
    return r * 180 * 60 / np.pi if arcmin else r
def alm2cl(alms, lmax=None, **kw):
    alms = np.asarray(alms)
    n = alms.shape[-1]
    L = int((-3 + np.sqrt(1 + 8 * n)) // 2)
    cl = np.zeros(L + 1)
    idx = 0
    for m in range(L + 1):
        seg = alms[idx: idx + L + 1 - m]
        w = 1.0 if m == 0 else 2.0
        cl[m:] += w * (seg.real ** 2 + seg.imag ** 2)
        idx += L + 1 - m
    return cl / (2 * np.arange(L + 1) + 1)
def read_map(path, *a, **k):
    return np.ones(12 * 256 * 256)
def ud_grade(m, nside_out, *a, **k):
    return np.ones(12 * nside_out * nside_out)
def map2alm(maps, lmax=None, iter=3, pol=True, **k):
    n = (lmax + 1) * (lmax + 2) // 2
    maps = np.asarray(maps)
    if maps.ndim == 2:
        return np.zeros((maps.shape[0], n), dtype=complex)
    return np.zeros(n, dtype=complex)
def alm2map(*a, **k):
    raise RuntimeError("SHT stub: not used by the full-sky fixtures")
def almxfl(alm, fl, inplace=False):
    out = alm if inplace else np.array(alm, copy=True)
    n = out.shape[-1]
    L = int((-3 + np.sqrt(1 + 8 * n)) // 2)
    idx = 0
    for m in range(L + 1):
        out[idx: idx + L + 1 - m] *= np.asarray(fl)[m:L + 1]
        idx += L + 1 - m
    return out
'''

QCINV_STUB = '''
class _Inert:
    def __init__(self, *a, **k): pass
class opfilt_tt:
    alm_filter_ninv = _Inert
class opfilt_pp:
    alm_filter_ninv = _Inert
class cd_solve:
    tr_cg = _Inert
    cache_mem = _Inert
class multigrid:
    pass
class util_alm:
    @staticmethod
    def lmax2nlm(l): return (l + 1) * (l + 2) // 2
'''

CLASSY_STUB = '''
class Class:
    def __init__(self, *a, **k): pass
'''


def make_stubs(tmp):
    os.makedirs(os.path.join(tmp, "healpy"), exist_ok=True)
    with open(os.path.join(tmp, "healpy", "__init__.py"), "w") as f:
        f.write(HEALPY_STUB)
    with open(os.path.join(tmp, "qcinv.py"), "w") as f:
        f.write(QCINV_STUB)
    with open(os.path.join(tmp, "classy.py"), "w") as f:
        f.write(CLASSY_STUB)


def import_reference(ref, tmp, L):
    os.environ.setdefault("SCRATCH", tmp)
    os.environ.setdefault("SLURM_ARRAY_TASK_ID", "0")
    if not hasattr(time, "clock"):
        time.clock = time.process_time
    sys.dont_write_bytecode = True
    sys.path.insert(0, ref)
    sys.path.insert(0, tmp)
    import config  # noqa
    config.L_MAX_SCALARS = L          # utils.real_to_complex reads it at call time
    import utils, CenteredGibbs, NonCenteredGibbs, ASIS  # noqa
    return types.SimpleNamespace(config=config, utils=utils, CG=CenteredGibbs,
                                 NCG=NonCenteredGibbs, ASIS=ASIS)


def problem(L, nside, seed=1234):
    """Small synthetic EB problem (SURVEY 8d fiducial, analytic spectra)."""
    rng = np.random.RandomState(seed)
    ell = np.arange(L + 1)
    dl_ee = np.where(ell >= 2, 10.0 * (np.maximum(ell, 1) / 100.0) ** 0.5, 0.0)
    dl_bb = np.where(ell >= 2, 0.01, 0.0)
    Npix = 12 * nside ** 2
    noise_pol = 0.2 ** 2
    fwhm = 0.5 * np.pi / 180 * 8      # wide beam so b_l varies at small L
    bl = np.exp(-0.5 * ell * (ell + 1) * (fwhm / np.sqrt(8 * np.log(2))) ** 2)
    # slot expansion
    slot_ell = [np.arange(L + 1)]
    for m in range(1, L + 1):
        slot_ell.append(np.repeat(np.arange(m, L + 1), 2))
    slot_ell = np.concatenate(slot_ell)
    fac = np.zeros(L + 1)
    fac[1:] = 2 * np.pi / (ell[1:] * (ell[1:] + 1))
    kappa = Npix / (4 * np.pi * noise_pol)
    d = {}
    for name, dl in (("EE", dl_ee), ("BB", dl_bb)):
        s_true = rng.normal(size=(L + 1) ** 2) * np.sqrt((dl * fac)[slot_ell])
        d[name] = bl[slot_ell] * s_true + rng.normal(size=(L + 1) ** 2) / np.sqrt(kappa)
    bins_ee = np.arange(0, L + 2)
    cut = (L * 2) // 3
    bins_bb = np.concatenate([np.arange(0, cut), np.array([cut + 1, cut + 3, L + 1])])
    bins_bb = np.unique(np.clip(bins_bb, 0, L + 1))
    blocks_ee = np.array([2, len(bins_ee)])
    kb = (len(bins_bb) - 1) // 2
    blocks_bb = np.concatenate([[2, kb], np.arange(kb + 1, len(bins_bb))])
    # proposal variances (config.py:119-132, 196-197)
    w = 4 * np.pi / Npix
    scale = np.array([((l * (l + 1)) ** 2 * 2 / (4 * np.pi ** 2 * (2 * l + 1))) for l in range(L + 1)])
    unb = (w * noise_pol / bl ** 2) ** 2 * scale

    def binned(b):
        return np.array([np.mean(unb[b[i]:b[i + 1]]) / (b[i + 1] - b[i]) for i in range(len(b) - 1)])
    pv = {"EE": binned(bins_ee)[2:], "BB": binned(bins_bb)[2:]}

    def bin_mean(dl, b):
        return np.array([np.mean(dl[b[i]:b[i + 1]]) for i in range(len(b) - 1)])
    init = {"EE": bin_mean(dl_ee, bins_ee), "BB": bin_mean(dl_bb, bins_bb)}
    return dict(L=L, nside=nside, Npix=Npix, noise_pol=noise_pol, noise_temp=40.0 ** 2,
                fwhm_deg=0.5 * 8, bl=bl, d_E=d["EE"], d_B=d["BB"],
                bins_EE=bins_ee, bins_BB=bins_bb, blocks_EE=blocks_ee, blocks_BB=blocks_bb,
                pv_EE=pv["EE"], pv_BB=pv["BB"], init_EE=init["EE"], init_BB=init["BB"],
                dl_EE=dl_ee, dl_BB=dl_bb)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..", "tests", "golden"))
    ap.add_argument("--L", type=int, default=16)
    ap.add_argument("--nside", type=int, default=8)
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    tmp = tempfile.mkdtemp(prefix="gs_stubs_")
    make_stubs(tmp)
    L, nside = args.L, args.nside
    R = import_reference(args.ref, tmp, L)
    P = problem(L, nside)
    Npix = P["Npix"]
    meta = dict(numpy=np.__version__, scipy=scipy.__version__, L=L, nside=nside)
    noise_temp = np.ones(Npix) * P["noise_temp"]
    noise_pol = np.ones(Npix) * P["noise_pol"]
    pix_map = {"EE": P["d_E"], "BB": P["d_B"], "Q": np.zeros(Npix), "U": np.zeros(Npix)}
    bins = {"EE": P["bins_EE"], "BB": P["bins_BB"]}
    blocks = {"EE": P["blocks_EE"], "BB": P["blocks_BB"]}
    pv = {"EE": P["pv_EE"], "BB": P["pv_BB"]}
    init = {"EE": P["init_EE"], "BB": P["init_BB"]}
    quiet = contextlib.redirect_stdout(io.StringIO())

    out = dict(P)
    out.update({"meta_" + k: v for k, v in meta.items()})

    # a1 / a3 / a4 / a5 -------------------------------------------------------
    rng = np.random.RandomState(7)
    dl_rand = rng.uniform(0.1, 5.0, size=L + 1)
    out["a1_dl"] = dl_rand
    out["a1_var"] = np.asarray(R.utils.generate_var_cl(dl_rand))
    x = rng.normal(size=(L + 1) ** 2)
    out["a3_real"] = x
    c = R.utils.real_to_complex(x)
    out["a3_cplx_re"], out["a3_cplx_im"] = c.real, c.imag
    out["a3_back"] = R.utils.complex_to_real(c)
    out["a5_binned"] = rng.uniform(size=len(P["bins_BB"]) - 1)
    out["a5_unfold"] = R.utils.unfold_bins(out["a5_binned"], P["bins_BB"])
    bl_map = np.concatenate([P["bl"], np.array([cl for m in range(1, L + 1) for cl in P["bl"][m:] for _ in range(2)])])

    # a7: centered full-sky CR ---------------------------------------------------
    all_dls = {"EE": P["dl_EE"], "BB": P["dl_BB"]}
    with quiet:
        cr = R.CG.PolarizedCenteredConstrainedRealization(pix_map, noise_temp, noise_pol, bl_map, L, Npix,
                                                            P["fwhm_deg"], mask_path=None)
    # reference computes its own bl_gauss from fwhm; use the same b_l everywhere
    out["bl_gauss_ref"] = cr.bl_gauss
    np.random.seed(101)
    with quiet:
        s7, acc7 = cr.sample_no_mask(all_dls)
    out["a7_seed"] = 101
    out["a7_E"], out["a7_B"], out["a7_accept"] = s7["EE"], s7["BB"], acc7

    # a8: non-centered all_sph CR -------------------------------------------------
    with quiet:
        ncr = R.NCG.PolarizedNonCenteredConstrainedRealization(pix_map, noise_temp, noise_pol, bl_map, L, Npix,
                                                               P["fwhm_deg"], mask_path=None, all_sph=True)
    np.random.seed(202)
    with quiet:
        s8, acc8 = ncr.sample_no_mask(all_dls)
    out["a8_seed"] = 202
    out["a8_E"], out["a8_B"], out["a8_accept"] = s8["EE"], s8["BB"], acc8

    # a13: centered C_l draw -----------------------------------------------------
    cls = R.CG.PolarizedCenteredClsSampler(pix_map, L, nside, bins, bl_map, noise_temp)
    np.random.seed(303)
    with quiet:
        d13 = cls.sample({"EE": s7["EE"].copy(), "BB": s7["BB"].copy()})
    out["a13_seed"] = 303
    out["a13_EE"], out["a13_BB"] = d13["EE"], d13["BB"]

    # a15: NC MH all_sph ---------------------------------------------------------
    mh = R.NCG.PolarizationNonCenteredClsSampler(pix_map, L, nside, bins, bl_map, noise_temp, noise_pol,
                                                 blocks, pv, n_iter=1, mask_path=None, all_sph=True)
    np.random.seed(404)
    with quiet:
        d15, a15 = mh.sample({"EE": s8["EE"].copy(), "BB": s8["BB"].copy()},
                             {"EE": init["EE"].copy(), "BB": init["BB"].copy()})
    out["a15_seed"] = 404
    out["a15_EE"], out["a15_BB"] = d15["EE"], d15["BB"]
    out["a15_acc_EE"], out["a15_acc_BB"] = np.array(a15["EE"]), np.array(a15["BB"])

    # a16: end-to-end drivers ----------------------------------------------------
    n_it = 6
    with quiet:
        ncg = R.NCG.NonCenteredGibbs(pix_map, noise_temp, noise_pol, P["fwhm_deg"], nside, L, Npix,
                                     proposal_variances=pv, metropolis_blocks=blocks, polarization=True,
                                     bins=bins, n_iter=n_it, mask_path=None, all_sph=True)
        np.random.seed(505)
        h, acc, _, _ = ncg.run({"EE": init["EE"].copy(), "BB": init["BB"].copy()})
    out["nc_seed"], out["nc_iters"] = 505, n_it
    out["nc_h_EE"], out["nc_h_BB"] = h["EE"], h["BB"]
    out["nc_acc_EE"], out["nc_acc_BB"] = acc["EE"], acc["BB"]

    with quiet:
        cg = R.CG.CenteredGibbs(pix_map, noise_temp, noise_pol, P["fwhm_deg"], nside, L, Npix, mask_path=None,
                                polarization=True, bins=bins, n_iter=n_it)
        csamp = cg.constrained_sampler
        csamp.sample = lambda all_dls, s_old=None: csamp.sample_no_mask(all_dls)
        np.random.seed(606)
        h, _, _, _ = cg.run({"EE": init["EE"].copy(), "BB": init["BB"].copy()})
    out["c_seed"], out["c_iters"] = 606, n_it
    out["c_h_EE"], out["c_h_BB"] = h["EE"], h["BB"]

    with quiet:
        asis = R.ASIS.ASIS(pix_map, noise_temp, noise_pol, P["fwhm_deg"], nside, L, Npix, pv,
                           metropolis_blocks=blocks, polarization=True, bins=bins, n_iter=n_it, mask_path=None,
                           all_sph=True)
        asamp = asis.constrained_sampler
        asamp.sample = lambda all_dls, s_old=None: asamp.sample_no_mask(all_dls)
        np.random.seed(707)
        res = asis.run({"EE": init["EE"].copy(), "BB": init["BB"].copy()})
    out["asis_seed"], out["asis_iters"] = 707, n_it
    out["asis_h_EE"], out["asis_h_BB"] = res[0]["EE"], res[0]["BB"]
    out["asis_acc_EE"], out["asis_acc_BB"] = res[1]["EE"], res[1]["BB"]

    path = os.path.join(args.out, f"reference_eb_L{L}.npz")
    np.savez(path, **{k: np.asarray(v) for k, v in out.items()})
    print("wrote", path, "keys:", len(out))


if __name__ == "__main__":
    main()
