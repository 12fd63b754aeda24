"""Puts the repository root (the parent of dropin/) on sys.path so the shims
find gibbssampler_amd without an install."""
import os
import sys

_root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _root not in sys.path:
    sys.path.append(_root)
