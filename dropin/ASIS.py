"""Drop-in for the reference's ASIS module (ASIS.py:16-233).
``from ASIS import ASIS`` (main_polarization.py:8).  No logic."""
import _gs_path  # noqa: F401,E402
from gibbssampler_amd.gibbs import ASIS  # noqa: F401

__all__ = ["ASIS"]
