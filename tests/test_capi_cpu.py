"""C-ABI checks that need no GPU: the library loads and exports every entry
point that include/gibbs_capi.h declares; the ctypes binding covers them."""
import os
import re
import ctypes

import pytest

from gibbssampler_amd import _capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "gibbs_capi.h")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(?:int|const char\*)\s+(gs_\w+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(_capi.LIB_PATH):
        from gibbssampler_amd.build import build
        build()
    return ctypes.CDLL(_capi.LIB_PATH)


def test_header_declares_the_hot_path():
    names = declared()
    for n in ("gs_plan_create", "gs_block_params", "gs_cr_sweep", "gs_cls_draw", "gs_nc_mh",
              "gs_step_centered", "gs_step_noncentered", "gs_step_asis", "gs_var_expand"):
        assert n in names


def test_every_declared_symbol_is_exported(lib):
    missing = [n for n in declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_covers_header():
    assert sorted(_capi.EXPORTED) == declared()


def test_abi_version_and_error_channel(lib):
    lib2 = _capi.load()
    assert lib2.gs_abi_version() == 1
    assert isinstance(lib2.gs_last_error(), bytes)


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(_capi.GibbsHipError):
        _capi.load(str(tmp_path / "nope.so"))


def _zero_args(argtypes):
    ints = (ctypes.c_int, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_longlong)
    return [0 if t in ints else (0.0 if t is ctypes.c_double else None) for t in argtypes]


def test_null_handles_are_errors_not_crashes(lib):
    """Every entry point taking a plan, SHT plan or masked context rejects a
    NULL handle with -1 and a message before any HIP call (the reference
    raises a Python exception where these return a status)."""
    lib2 = _capi.load()
    checked = 0
    for name, _, argtypes in _capi._SIGS:
        if not argtypes or argtypes[0] is not ctypes.c_void_p or name.endswith("_destroy"):
            continue
        rc = getattr(lib2, name)(*_zero_args(argtypes))
        assert rc == -1, name
        assert b"null" in lib2.gs_last_error(), (name, lib2.gs_last_error())
        checked += 1
    assert checked >= 30
    for name in ("gs_plan_destroy", "gs_sht_destroy", "gs_masked_destroy"):
        assert getattr(lib2, name)(None) == 0          # destroying NULL is a no-op


def test_stateless_helpers_validate_before_launch(lib):
    """Sizes and buffers are checked before any launch; an empty batch is a
    no-op (no kernel, no GPU needed)."""
    lib2 = _capi.load()
    for name in ("gs_var_expand", "gs_real_to_complex", "gs_complex_to_real"):
        fn = getattr(lib2, name)
        assert fn(-1, 1, None, None, None) == -1
        assert b"out of range" in lib2.gs_last_error()
        assert fn(8, 1, None, None, None) == -1
        assert b"null" in lib2.gs_last_error()
        assert fn(8, 0, None, None, None) == 0
    assert lib2.gs_remove_monopole_dipole(8, 0, None, None) == 0
    assert lib2.gs_remove_monopole_dipole(8, -2, None, None) == -1
    assert lib2.gs_alm2cl(8, 0, None, None, None, None) == 0
    assert lib2.gs_alm2cl(8, 2, None, None, None, None) == -1
    assert lib2.gs_unfold_bins(0, None, None, 5, None, None) == 0
    assert lib2.gs_unfold_bins(2, None, None, 5, None, None) == -1
    assert lib2.gs_synalm(-1, 3, None, None, None, None, None) == -1


def test_create_rejects_bad_sizes(lib):
    lib2 = _capi.load()
    out = ctypes.c_void_p()
    assert lib2.gs_plan_create(None, ctypes.byref(out)) == -1
    d = _capi.GsModelDesc()
    for lmax, nf, nch, msg in ((1, 3, 1, b"lmax"), (64, 4, 1, b"nfields"), (64, 3, 0, b"nchains")):
        d.lmax, d.nfields, d.nchains = lmax, nf, nch
        assert lib2.gs_plan_create(ctypes.byref(d), ctypes.byref(out)) == -1
        assert msg in lib2.gs_last_error()
    assert lib2.gs_sht_create(3, 6, ctypes.byref(out)) == -1
    assert b"power of two" in lib2.gs_last_error()
    assert lib2.gs_sht_create(8, 40, ctypes.byref(out)) == -1
    assert b"lmax" in lib2.gs_last_error()
    assert lib2.gs_masked_create(None, None, None, ctypes.byref(out)) == -1
    assert not out.value


def test_library_options_registry():
    """gs_option_set / gs_option_get (the library reads no environment
    variables): a registered name round-trips and unsets; an unknown name is an
    error with a message, not a silent no-op."""
    _capi.load()
    assert _capi.get_option("GS_SWEEP_TW") is None
    with _capi.options(GS_SWEEP_TW=2):
        assert _capi.get_option("GS_SWEEP_TW") == "2"
    assert _capi.get_option("GS_SWEEP_TW") is None
    with pytest.raises(_capi.GibbsHipError, match="unknown option"):
        _capi.set_option("GS_NO_SUCH_KNOB", 1)
    assert _capi.get_option("GS_NO_SUCH_KNOB") is None
    src = "".join(open(os.path.join(ROOT, "gibbssampler_amd", "csrc", f)).read()
                  for f in os.listdir(os.path.join(ROOT, "gibbssampler_amd", "csrc")))
    assert "getenv" not in src
