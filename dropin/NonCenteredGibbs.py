"""Drop-in for the reference's NonCenteredGibbs module (NonCenteredGibbs.py:449-582).
``from NonCenteredGibbs import NonCenteredGibbs`` (main_polarization.py:7).  No logic."""
import _gs_path  # noqa: F401,E402
from gibbssampler_amd.gibbs import (NonCenteredGibbs, NonCenteredClsSampler,  # noqa: F401
                                    NonCenteredConstrainedRealization)

__all__ = ["NonCenteredGibbs", "NonCenteredClsSampler", "NonCenteredConstrainedRealization"]
