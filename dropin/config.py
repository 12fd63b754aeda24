"""Drop-in for the reference's global ``config`` module (config.py:1-225):
``import config`` (main_polarization.py:2) gets the module-level names of
gibbssampler_amd.config (N_side 256 / l_max 512 defaults, Planck BB bins,
Metropolis blocks, proposal variances, beam).  No logic."""
import _gs_path  # noqa: F401,E402
import sys as _sys

from gibbssampler_amd import config as _cfg

_sys.modules[__name__] = _cfg
