"""Drop-in for the reference's CenteredGibbs module (CenteredGibbs.py:859-876).

Put ``dropin/`` on ``sys.path`` in place of the reference checkout and
``from CenteredGibbs import CenteredGibbs`` (main_polarization.py:9) resolves
to the MI355X implementation.  No logic lives here."""
import _gs_path  # noqa: F401,E402
from gibbssampler_amd.gibbs import (CenteredGibbs, CenteredClsSampler,  # noqa: F401
                                    CenteredConstrainedRealization)

__all__ = ["CenteredGibbs", "CenteredClsSampler", "CenteredConstrainedRealization"]
