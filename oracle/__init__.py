"""CPU oracle for the Gibbs hot path -- TEST INFRASTRUCTURE ONLY.

This package is a numpy restatement of the reference's per-iteration algebra
(Gabriel-Ducrocq/GibbsSampler: utils.py, CenteredGibbs.py, NonCenteredGibbs.py,
ASIS.py, ClsSampler.py, variance_expension.pyx) plus the build's own
specification of the TEB (T, E, B with TE coupling) generalisation.

Rules (DESIGN.md "Oracle"):
  * Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
    ``cpu_baseline`` leg may import anything under ``oracle/``.
  * The product package ``gibbssampler_amd`` never imports it; the HIP path
    fails loudly when its extension is missing.
  * Parity pin: the EB (EE/BB) subset is checked against golden vectors that
    ``tools/gen_golden.py`` produced by importing the reference's own Python
    in the build container (``tests/golden/*.npz``).  The TEB extension and
    the counter-based (Philox) native RNG streams are build-specified; they
    reduce exactly to the pinned EB path when TT = TE = 0.
"""
