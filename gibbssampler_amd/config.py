"""config.py surface of the reference (config.py:19-225) without its import-time
side effects (no $SCRATCH / $SLURM_ARRAY_TASK_ID, no FITS mask read).

Names are kept so that callers written against the reference find them.
The default resolution is the reference's (NSIDE = 256, L = 512); use
``make_config(nside)`` for another one.
"""
import math
import os
from dataclasses import dataclass, field

import numpy as np

from .problem import BINS_BB_512, gauss_beam, default_blocks, proposal_variances


# cosmological parameter prior (config.py:10-12); the theory spectra they feed
# (utils.generate_cls through CLASS) are out of scope
COSMO_PARAMS_NAMES = ["n_s", "omega_b", "omega_cdm", "100*theta_s", "ln10^{10}A_s", "tau_reio"]
COSMO_PARAMS_MEAN_PRIOR = np.array([0.9665, 0.02242, 0.11933, 1.04101, 3.047, 0.0561])
COSMO_PARAMS_SIGMA_PRIOR = np.array([0.0038, 0.00014, 0.00091, 0.00029, 0.014, 0.0071])
# config.py:205-207 sets it from preliminary chains (non-preliminary runs only)
starting_point = None


@dataclass
class GibbsConfig:
    NSIDE: int = 256
    noise_covar_temp: float = 40.0 ** 2          # config.py:36
    noise_covar_pol: float = 0.2 ** 2            # config.py:38
    beam_fwhm: float = 0.5                       # config.py:87 (degrees)
    mask_path: str = None                        # config.py:26 (Planck mask absent offline)
    preliminary_run: bool = True                 # config.py:161
    scratch_path: str = field(default_factory=lambda: os.environ.get("SCRATCH", "."))
    slurm_task_id: str = field(default_factory=lambda: os.environ.get("SLURM_ARRAY_TASK_ID", "0"))

    def __post_init__(self):
        self.Npix = 12 * self.NSIDE ** 2
        self.L_MAX_SCALARS = int(2 * self.NSIDE)
        L = self.L_MAX_SCALARS
        self.var_noise_temp = np.ones(self.Npix) * self.noise_covar_temp
        self.var_noise_pol = np.ones(self.Npix) * self.noise_covar_pol
        bins_bb = BINS_BB_512.copy() if L == 512 else np.arange(0, L + 2)
        self.bins = {"EE": np.arange(0, L + 2), "BB": bins_bb}
        self.blocks = default_blocks(L, self.bins)
        self.metropolis_blocks_gibbs_nc = self.blocks
        self.metropolis_blocks_gibbs_asis = self.blocks
        self.rescaling_map2alm = self.Npix / (4 * np.pi)      # config.py:72
        self.w = 4 * np.pi / self.Npix                        # config.py:73
        self.fwhm_radians = (np.pi / 180) * self.beam_fwhm
        self.bl_gauss = gauss_beam(self.fwhm_radians, L)
        self.bl_map = np.concatenate([self.bl_gauss, np.array(
            [cl for m in range(1, L + 1) for cl in self.bl_gauss[m:] for _ in range(2)])])
        self.mask_inversion = np.ones((L + 1) ** 2, dtype=bool)      # cp38 config, src line 56-58
        self.mask_inversion[[0, 1, L + 1, L + 2]] = False
        self.proposal_variances_nc_polarized = proposal_variances(L, self.NSIDE, self.bins, self.bl_gauss,
                                                                  self.noise_covar_pol, self.noise_covar_temp)

    def compute_init_values_pol(self, unbinned_vars, pol):
        """config.py:93-104."""
        b = self.bins[pol]
        return np.array([np.mean(unbinned_vars[b[i]:b[i + 1]]) / (b[i + 1] - b[i]) for i in range(len(b) - 1)])


def make_config(nside=256, **kw):
    return GibbsConfig(NSIDE=nside, **kw)


_default = GibbsConfig()
# module-level names, as `import config; config.NSIDE` in the reference
for _k, _v in vars(_default).items():
    globals()[_k] = _v
generate_var_cl = None   # the reference's config.generate_var_cl is utils.generate_var_cl (see utils)
del _k, _v, math
