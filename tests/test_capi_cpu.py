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
