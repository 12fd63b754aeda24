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
