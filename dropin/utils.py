"""Drop-in for the reference's ``utils`` module (utils.py:49-162):
``import utils`` (main_polarization.py:1) gets gibbssampler_amd.utils
(generate_var_cl, real_to_complex, complex_to_real, unfold_bins,
adjoint_synthesis_hp on the device).  No logic."""
import _gs_path  # noqa: F401,E402
import sys as _sys

from gibbssampler_amd import utils as _utils

_sys.modules[__name__] = _utils
