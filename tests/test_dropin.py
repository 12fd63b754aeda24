"""The unchanged-caller drop-in: with ``dropin/`` on
sys.path in place of the reference checkout, the reference-module imports of
main_polarization.py (lines 1-2, 7-9) resolve to this package, its constructor
calls (main_polarization.py:109-126) bind to the classes' signatures, and every
``config.<name>`` / ``<sampler>.constrained_sampler.<name>`` it reads exists.

The caller is read from /root/reference when it is present (parsed with ast,
as text; nothing of it is executed or copied); otherwise the test restates
only the keyword names of those calls.  CPU only: binding checks signatures,
nothing is constructed on a device."""
import ast
import importlib
import inspect
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DROPIN = os.path.join(ROOT, "dropin")
CALLER = "/root/reference/main_polarization.py"
REF_MODULES = ("utils", "config", "NonCenteredGibbs", "ASIS", "CenteredGibbs")

# keyword names of main_polarization.py:109-126 (fallback when the caller is absent)
_FALLBACK_CALLS = {
    "CenteredGibbs": [8, ["mask_path", "polarization", "bins", "n_iter", "rj_step", "gibbs_cr", "overrelaxation",
                          "ula"]],
    "NonCenteredGibbs": [7, ["mask_path", "polarization", "bins", "n_iter", "proposal_variances",
                             "metropolis_blocks", "all_sph"]],
    "ASIS": [7, ["mask_path", "polarization", "bins", "n_iter", "proposal_variances", "metropolis_blocks",
                 "rj_step", "all_sph", "gibbs_cr", "n_gibbs", "overrelaxation"]],
}


@pytest.fixture
def dropin_modules():
    saved = {k: sys.modules.pop(k) for k in REF_MODULES + ("_gs_path",) if k in sys.modules}
    sys.path.insert(0, DROPIN)
    try:
        yield {m: importlib.import_module(m) for m in REF_MODULES}
    finally:
        sys.path.remove(DROPIN)
        for k in REF_MODULES + ("_gs_path",):
            sys.modules.pop(k, None)
        sys.modules.update(saved)


def _caller_tree():
    if not os.path.exists(CALLER):
        return None
    import warnings
    with open(CALLER) as f, warnings.catch_warnings():
        warnings.simplefilter("ignore", DeprecationWarning)     # the caller's docstring escapes
        return ast.parse(f.read())


def _constructor_calls(tree):
    """(class name, positional count, keyword names) of every call of the
    three sampler classes in the caller."""
    if tree is None:
        return [(k, n, kw) for k, (n, kw) in _FALLBACK_CALLS.items()]
    out = []
    for node in ast.walk(tree):
        if isinstance(node, ast.Call) and isinstance(node.func, ast.Name) and \
                node.func.id in ("CenteredGibbs", "NonCenteredGibbs", "ASIS"):
            out.append((node.func.id, len(node.args), [k.arg for k in node.keywords]))
    return out


def test_reference_imports_resolve_to_this_package(dropin_modules):
    import gibbssampler_amd.config as gcfg
    import gibbssampler_amd.gibbs as gg
    import gibbssampler_amd.utils as gutils
    m = dropin_modules
    assert m["config"] is gcfg and m["utils"] is gutils
    assert m["CenteredGibbs"].CenteredGibbs is gg.CenteredGibbs
    assert m["NonCenteredGibbs"].NonCenteredGibbs is gg.NonCenteredGibbs
    assert m["ASIS"].ASIS is gg.ASIS
    tree = _caller_tree()
    if tree is not None:
        for node in ast.walk(tree):
            if isinstance(node, ast.ImportFrom) and node.module in REF_MODULES:
                for a in node.names:
                    assert hasattr(m[node.module], a.name), (node.module, a.name)
            elif isinstance(node, ast.Import):
                for a in node.names:
                    if a.name in REF_MODULES:
                        assert a.name in m


def test_constructor_calls_bind(dropin_modules):
    m = dropin_modules
    calls = _constructor_calls(_caller_tree())
    assert {c[0] for c in calls} == {"CenteredGibbs", "NonCenteredGibbs", "ASIS"}
    for name, npos, kws in calls:
        cls = getattr(m[name], name)
        sig = inspect.signature(cls.__init__)
        sig.bind(None, *([0] * npos), **{k: 0 for k in kws})


def test_config_and_attribute_reads_exist(dropin_modules):
    cfg = dropin_modules["config"]
    tree = _caller_tree()
    names = {"NSIDE", "L_MAX_SCALARS", "Npix", "beam_fwhm", "mask_path", "bins", "blocks",
             "proposal_variances_nc_polarized", "noise_covar_temp", "noise_covar_pol", "bl_gauss",
             "preliminary_run", "starting_point", "scratch_path", "slurm_task_id", "COSMO_PARAMS_MEAN_PRIOR",
             "fwhm_radians", "var_noise_temp", "var_noise_pol"}
    if tree is not None:
        names |= {n.attr for n in ast.walk(tree) if isinstance(n, ast.Attribute) and isinstance(n.value, ast.Name)
                  and n.value.id == "config"}
    missing = sorted(n for n in names if not hasattr(cfg, n))
    assert not missing, missing
    assert cfg.NSIDE == 256 and cfg.L_MAX_SCALARS == 512 and len(cfg.bins["BB"]) == 413
    # main_polarization.py:180-182 reads these off the ASIS sampler and its step object
    import types
    import gibbssampler_amd.gibbs as gg
    owner = types.SimpleNamespace(lmax=16, nside=8, Npix=768, bl_map=None, bl_gauss=None, pix_map=None,
                                  gibbs_cr=True)
    step = gg._StepBase(owner)
    assert step.pcg_accuracy == 1.0e-5 and step.gibbs_cr is True and step.n_gibbs == 1
    assert "rj_step" in inspect.signature(dropin_modules["ASIS"].ASIS.__init__).parameters
