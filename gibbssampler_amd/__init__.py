"""gibbssampler_amd -- MI355X-native Gibbs hot path for CMB power-spectrum sampling.

Drop-in for the CenteredGibbs / NonCenteredGibbs / ASIS class surface of
Gabriel-Ducrocq/GibbsSampler, with the per-iteration hot path (constrained
realisation, C_l draw, per-l expansion) in hand-written gfx950 HIP kernels
behind a ctypes C-ABI (include/gibbs_capi.h).
"""
__version__ = "0.1.0"

from . import _capi  # noqa: F401
