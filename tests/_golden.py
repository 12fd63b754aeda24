"""Helpers to build oracle models from the reference-generated golden fixtures."""
import os

import numpy as np

from oracle import harmonic as H

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(L=16):
    return dict(np.load(os.path.join(GOLDEN, f"reference_eb_L{L}.npz")))


def model_from(g):
    L = int(g["L"])
    return H.Model(L=L, nside=int(g["nside"]), nfields=2, bl=g["bl"],
                   noise_var=[float(g["noise_pol"])] * 2,
                   bins={"EE": g["bins_EE"], "BB": g["bins_BB"]},
                   blocks={"EE": g["blocks_EE"], "BB": g["blocks_BB"]},
                   proposal_variances={"EE": g["pv_EE"], "BB": g["pv_BB"]},
                   d_alm=np.stack([g["d_E"], g["d_B"]]))


def init_of(g):
    return {"EE": g["init_EE"].copy(), "BB": g["init_BB"].copy()}


def scale_data(L, nside, seed, fwhm_deg=0.5, noise_pol=0.2 ** 2):
    """Synthetic EB harmonic data at the reference's default configuration
    (config.py:19-21: N_side 256, L 512; beam config.py:87-90; noise
    config.py:38), d = b s_true + n with the SURVEY 8d fiducial spectra.  Used
    by tools/gen_golden_scale.py to drive the reference and by the tests to
    regenerate the same d (numpy RandomState, so the fixture holds no maps)."""
    rng = np.random.RandomState(seed)
    ell = np.arange(L + 1)
    dl_ee = np.where(ell >= 2, 10.0 * (np.maximum(ell, 1) / 100.0) ** 0.5, 0.0)
    dl_bb = np.where(ell >= 2, 0.01, 0.0)
    Npix = 12 * nside ** 2
    bl = H.gauss_beam(np.radians(fwhm_deg), L)
    sl = H.slot_ell(L)
    kappa = Npix / (4 * np.pi * noise_pol)
    fac = H.dl_to_cl_factor(L)
    d = {}
    for name, dl in (("EE", dl_ee), ("BB", dl_bb)):
        s_true = rng.normal(size=(L + 1) ** 2) * np.sqrt((dl * fac)[sl])
        d[name] = bl[sl] * s_true + rng.normal(size=(L + 1) ** 2) / np.sqrt(kappa)
    return {"d_E": d["EE"], "d_B": d["BB"], "dl_EE": dl_ee, "dl_BB": dl_bb, "bl": bl, "Npix": Npix,
            "noise_pol": noise_pol}


def scale_model(g):
    """Oracle model of the scale fixture (data regenerated from its seed)."""
    L, nside = int(g["L"]), int(g["nside"])
    D = scale_data(L, nside, int(g["data_seed"]))
    m = H.Model(L=L, nside=nside, nfields=2, bl=g["bl"], noise_var=[float(g["noise_pol"])] * 2,
                bins={"EE": g["bins_EE"], "BB": g["bins_BB"]},
                blocks={"EE": g["blocks_EE"], "BB": g["blocks_BB"]},
                proposal_variances={"EE": g["pv_EE"], "BB": g["pv_BB"]},
                d_alm=np.stack([D["d_E"], D["d_B"]]))
    return m, D
