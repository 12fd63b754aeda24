"""ctypes binding of libgibbs_hip.so (include/gibbs_capi.h).

This is the reference-side binding a maintainer would add to
Gabriel-Ducrocq/GibbsSampler: plain ctypes over the C-ABI,
device pointers from torch tensors, the HIP stream from
``torch.cuda.current_stream().cuda_stream``.  There is no CPU fallback: if the
library is missing or fails to load, every entry point raises.
"""
import contextlib
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GIBBS_HIP_LIB", os.path.join(_HERE, "libgibbs_hip.so"))

GS_MODE_CENTERED = 0
GS_MODE_NONCENTERED = 1
GS_QUIRK_ASIS_RECENTRE_CENTERED = 1
GS_NPARAM = 10
GS_ALM_REAL = 0
GS_ALM_COMPLEX = 1
GS_MCR_AUX, GS_MCR_OVERRELAX, GS_MCR_MALA, GS_MCR_AUX_MALA = 0, 1, 2, 3
NSTAT = {1: 2, 2: 4, 3: 8}

c_int_p = ctypes.POINTER(ctypes.c_int)
c_double_p = ctypes.POINTER(ctypes.c_double)


class GsModelDesc(ctypes.Structure):
    _fields_ = [
        ("lmax", ctypes.c_int),
        ("nside", ctypes.c_int),
        ("nfields", ctypes.c_int),
        ("nchains", ctypes.c_int),
        ("chain0", ctypes.c_int),
        ("quirks", ctypes.c_int),
        ("n_iter_metropolis", ctypes.c_int),
        ("bl", c_double_p),
        ("noise_var", c_double_p),
        ("bins", c_int_p * 4),
        ("nbin_edges", ctypes.c_int * 4),
        ("blocks", c_int_p * 4),
        ("nblock_edges", ctypes.c_int * 4),
        ("prop_var", c_double_p * 4),
    ]


class GsMaskedDesc(ctypes.Structure):
    _fields_ = [
        ("lmax", ctypes.c_int),
        ("nside", ctypes.c_int),
        ("nfields", ctypes.c_int),
        ("bl", c_double_p),
        ("n_gibbs", ctypes.c_int),
        ("alpha", ctypes.c_double),
        ("tau", ctypes.c_double),
        ("noise_pol0", ctypes.c_double),
        ("mu_eps", ctypes.c_double),
        ("adj_iter", ctypes.c_int),
        ("nchains", ctypes.c_int),
        ("sht_mode", ctypes.c_int),
    ]


class GibbsHipError(RuntimeError):
    pass


_lib = None

# (name, restype, argtypes)
_VP = ctypes.c_void_p
_SIGS = [
    ("gs_abi_version", ctypes.c_int, []),
    ("gs_last_error", ctypes.c_char_p, []),
    ("gs_option_set", ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p]),
    ("gs_option_get", ctypes.c_char_p, [ctypes.c_char_p]),
    ("gs_plan_create", ctypes.c_int, [ctypes.POINTER(GsModelDesc), ctypes.POINTER(_VP)]),
    ("gs_plan_destroy", ctypes.c_int, [_VP]),
    ("gs_plan_info", ctypes.c_int, [_VP, c_int_p, c_int_p, c_int_p, c_int_p]),
    ("gs_plan_sweep_info", ctypes.c_int, [_VP, c_int_p, c_int_p]),
    ("gs_var_expand", ctypes.c_int, [ctypes.c_int, ctypes.c_int, _VP, _VP, _VP]),
    ("gs_real_to_complex", ctypes.c_int, [ctypes.c_int, ctypes.c_int, _VP, _VP, _VP]),
    ("gs_complex_to_real", ctypes.c_int, [ctypes.c_int, ctypes.c_int, _VP, _VP, _VP]),
    ("gs_remove_monopole_dipole", ctypes.c_int, [ctypes.c_int, ctypes.c_int, _VP, _VP]),
    ("gs_alm2cl", ctypes.c_int, [ctypes.c_int, ctypes.c_int, _VP, _VP, _VP, _VP]),
    ("gs_unfold_bins", ctypes.c_int, [ctypes.c_int, _VP, _VP, ctypes.c_int, _VP, _VP]),
    ("gs_block_params", ctypes.c_int, [_VP, ctypes.c_int, _VP, _VP, _VP]),
    ("gs_cr_sweep", ctypes.c_int, [_VP, _VP, _VP, _VP, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                   _VP, _VP, _VP]),
    ("gs_sweep_stats", ctypes.c_int, [_VP, _VP, _VP, _VP, _VP]),
    ("gs_cls_draw", ctypes.c_int, [_VP, _VP, _VP, ctypes.c_uint64, ctypes.c_uint32, _VP, _VP]),
    ("gs_nc_mh", ctypes.c_int, [_VP, _VP, _VP, _VP, _VP, ctypes.c_uint64, ctypes.c_uint32, _VP, _VP]),
    ("gs_stats_to_noncentered", ctypes.c_int, [_VP, _VP, _VP, _VP]),
    ("gs_recentre", ctypes.c_int, [_VP, _VP, _VP, _VP, _VP]),
    ("gs_step_centered", ctypes.c_int, [_VP, _VP, _VP, _VP, _VP, _VP, ctypes.c_uint64, ctypes.c_uint32, _VP]),
    ("gs_step_asis_fused", ctypes.c_int, [_VP, _VP, _VP, _VP, ctypes.c_uint64, ctypes.c_uint32, _VP, _VP, ctypes.c_int,
                                          _VP, ctypes.c_int, _VP]),
    ("gs_step_centered_fused", ctypes.c_int, [_VP, _VP, _VP, _VP, ctypes.c_uint64, ctypes.c_uint32, _VP, ctypes.c_int,
                                              _VP]),
    ("gs_step_noncentered", ctypes.c_int, [_VP, _VP, _VP, _VP, _VP, _VP, _VP, ctypes.c_uint64, ctypes.c_uint32,
                                           _VP, _VP]),
    ("gs_nc_prologue", ctypes.c_int, [_VP, _VP, _VP, ctypes.c_uint64, ctypes.c_uint32, _VP]),
    ("gs_nc_sweep", ctypes.c_int, [_VP, _VP, _VP, _VP, _VP, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, _VP]),
    ("gs_nc_finish", ctypes.c_int, [_VP, _VP]),
    ("gs_nc_decide", ctypes.c_int, [_VP, _VP, _VP, ctypes.c_uint64, ctypes.c_uint32, _VP, _VP]),
    ("gs_nc_decide_fused", ctypes.c_int, [_VP, _VP, ctypes.c_uint64, ctypes.c_uint32, _VP, _VP, ctypes.c_int, _VP]),
    ("gs_step_asis", ctypes.c_int, [_VP, _VP, _VP, _VP, _VP, _VP, _VP, _VP, ctypes.c_uint64, ctypes.c_uint32,
                                    _VP, _VP, ctypes.c_int, _VP]),
    ("gs_iteration_counter", ctypes.c_int, [_VP, ctypes.c_int, ctypes.c_uint32]),
    ("gs_graph_step", ctypes.c_int, [_VP, ctypes.c_uint32, ctypes.c_uint32]),
    ("gs_advance_iteration", ctypes.c_int, [_VP, _VP]),
    ("gs_record_trace", ctypes.c_int, [_VP, _VP, _VP, ctypes.c_int, ctypes.c_uint32, _VP]),
    ("gs_sweep_timing", ctypes.c_int, [_VP, ctypes.c_int, c_double_p, c_int_p]),
    ("gs_sht_create", ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.POINTER(_VP)]),
    ("gs_sht_destroy", ctypes.c_int, [_VP]),
    ("gs_sht_info", ctypes.c_int, [_VP, c_int_p, c_int_p, ctypes.POINTER(ctypes.c_longlong),
                                   ctypes.POINTER(ctypes.c_longlong)]),
    ("gs_sht_alm2map", ctypes.c_int, [_VP, ctypes.c_int, ctypes.c_int, _VP, _VP, _VP]),
    ("gs_sht_map2alm", ctypes.c_int, [_VP, ctypes.c_int, ctypes.c_int, _VP, _VP, ctypes.c_int, _VP]),
    ("gs_sht_alm2map_beamed", ctypes.c_int, [_VP, ctypes.c_int, _VP, _VP, _VP, _VP]),
    ("gs_sht_map2alm_weighted", ctypes.c_int, [_VP, ctypes.c_int, _VP, _VP, _VP, _VP]),
    ("gs_sht_reserve", ctypes.c_int, [_VP, ctypes.c_int, _VP]),
    ("gs_sht_set_mfma", ctypes.c_int, [_VP, ctypes.c_int]),
    ("gs_sht_mfma_info", ctypes.c_int, [_VP, c_int_p, ctypes.POINTER(ctypes.c_longlong)]),
    ("gs_sht_alm2map_batch", ctypes.c_int, [_VP, ctypes.c_int, ctypes.c_int, ctypes.c_int, _VP, _VP, _VP, _VP]),
    ("gs_sht_apply_weighted_batch", ctypes.c_int, [_VP, ctypes.c_int, ctypes.c_int, _VP, _VP, _VP, _VP, _VP, _VP]),
    ("gs_sht_map2alm_batch", ctypes.c_int, [_VP, ctypes.c_int, ctypes.c_int, ctypes.c_int, _VP, _VP, _VP,
                                            ctypes.c_int, _VP]),
    ("gs_masked_create", ctypes.c_int, [ctypes.POINTER(GsMaskedDesc), _VP, _VP, ctypes.POINTER(_VP)]),
    ("gs_masked_destroy", ctypes.c_int, [_VP]),
    ("gs_masked_ring_classes", ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_int)]),
    ("gs_masked_info", ctypes.c_int, [_VP, c_double_p, _VP]),
    ("gs_masked_nchains", ctypes.c_int, [_VP]),
    ("gs_masked_sht_tables", ctypes.c_int, [_VP]),
    ("gs_masked_gradient", ctypes.c_int, [_VP, _VP, _VP, _VP, _VP, _VP]),
    ("gs_masked_pcg_rhs", ctypes.c_int, [_VP, _VP, _VP, _VP, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, _VP,
                                         _VP]),
    ("gs_masked_pcg_solve", ctypes.c_int, [_VP, _VP, _VP, _VP, ctypes.c_int, ctypes.c_double, ctypes.c_int, c_int_p,
                                           c_double_p, _VP]),
    ("gs_masked_pcg_info", ctypes.c_int, [_VP, c_int_p]),
    ("gs_masked_pcg_info2", ctypes.c_int, [_VP, c_int_p, c_int_p]),
    ("gs_masked_pcg_work", ctypes.c_int, [_VP, ctypes.POINTER(ctypes.c_longlong)]),
    ("gs_masked_pcg_apply", ctypes.c_int, [_VP, _VP, _VP, _VP, _VP]),
    ("gs_masked_rj_accept", ctypes.c_int, [_VP, _VP, _VP, _VP, _VP, _VP, ctypes.c_uint64, ctypes.c_uint32,
                                           ctypes.c_int, _VP, _VP, _VP]),
    ("gs_masked_center", ctypes.c_int, [_VP, _VP, ctypes.c_int, _VP, _VP, _VP]),
    ("gs_masked_nc_loglik", ctypes.c_int, [_VP, _VP, _VP, _VP, _VP]),
    ("gs_masked_pixel_mh", ctypes.c_int, [_VP, ctypes.c_int, ctypes.c_int, ctypes.c_int] + [_VP] * 13),
    ("gs_masked_tt_fullsky", ctypes.c_int, [_VP, ctypes.c_int, _VP, _VP, _VP, ctypes.c_uint64, ctypes.c_uint32,
                                             ctypes.c_int, _VP, _VP]),
    ("gs_synalm", ctypes.c_int, [ctypes.c_int, ctypes.c_int, _VP, _VP, _VP, _VP, _VP]),
    ("gs_mh_propose", ctypes.c_int, [_VP, _VP, _VP, ctypes.c_uint64, ctypes.c_uint32, _VP, _VP, _VP, _VP]),
    ("gs_masked_cr", ctypes.c_int, [_VP, ctypes.c_int, _VP, _VP, _VP, _VP, _VP, _VP, _VP, ctypes.c_uint64,
                                    ctypes.c_uint32, ctypes.c_int, _VP, _VP, _VP]),
]

EXPORTED = [n for n, _, _ in _SIGS]


def load(path=None, allow_missing=False):
    """Load the HIP library (raises GibbsHipError when absent).  allow_missing:
    tolerate entry points an older build lacks (the A/B tools load earlier
    builds side by side; the product path never passes it)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise GibbsHipError(f"libgibbs_hip.so not found at {p}: run __graft_entry__.build() "
                            "(there is no CPU fallback)")
    lib = ctypes.CDLL(p)
    for name, res, args in _SIGS:
        if allow_missing and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.gs_abi_version() != 1:
        raise GibbsHipError("ABI version mismatch")
    _lib = lib
    return lib


def check(rc, what="gibbs_hip"):
    if rc != 0:
        msg = _lib.gs_last_error().decode() if _lib is not None else "?"
        raise GibbsHipError(f"{what} failed: {msg}")


def set_option(name, value):
    """Library option (include/gibbs_capi.h gs_option_set): read when a plan,
    SHT or masked context is created; value None unsets it."""
    lib = load()
    v = None if value is None else str(value).encode()
    check(lib.gs_option_set(name.encode(), v), f"gs_option_set({name})")


def get_option(name):
    r = load().gs_option_get(name.encode())
    return None if r is None else r.decode()


@contextlib.contextmanager
def options(**kw):
    """Set library options for the body (restored afterwards), e.g.
    ``with options(GS_SWEEP_TW=2): BatchedRunner(...)``."""
    old = {k: get_option(k) for k in kw}
    try:
        for k, v in kw.items():
            set_option(k, v)
        yield
    finally:
        for k, v in old.items():
            set_option(k, v)


def ptr(t):
    """Device pointer of a torch tensor (None -> NULL)."""
    if t is None:
        return None
    if not t.is_contiguous():
        raise GibbsHipError("tensor must be contiguous")
    return ctypes.c_void_p(t.data_ptr())


def stream_ptr(stream=None):
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


# ---------------------------------------------------------------------------------------
# capture-safe teardown
# ---------------------------------------------------------------------------------------
# A destructor that runs while a hipGraph capture is open (a reference dropped
# inside the captured code, or a cyclic collection there) must not call HIP:
# hipFree / hipGraphExecDestroy / hipStreamDestroy are illegal during capture
# and invalidate it (the intermittent fault of r03, commit 2ac910f).  Objects
# that own device resources hand them to ``release`` / ``park``: outside a
# capture they are freed at once; inside one they wait in the graveyard until
# the outermost capture of samplers._capture has ended (``end_capture``).
_GRAVEYARD = []
_CAPTURE_DEPTH = [0]


def capturing():
    """True while one of this package's captures is open, or while the current
    stream is being captured by anyone (torch.cuda.graph used directly)."""
    if _CAPTURE_DEPTH[0] > 0:
        return True
    try:
        import torch
        return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
    except Exception:       # interpreter shutdown
        return False


def _drain():
    """Run the deferred releases (no capture open)."""
    while _GRAVEYARD:
        fn, h = _GRAVEYARD.pop()
        if fn is not None:
            try:
                fn(h)
            except Exception:
                pass


def release(fn, handle):
    """Call fn(handle) now, or after the open capture ends."""
    if capturing():
        _GRAVEYARD.append((fn, handle))
    else:
        fn(handle)


def park(obj):
    """Keep obj (e.g. a dying runner's graphs, streams and tensors) alive until
    the open capture ends; False when no capture is open (nothing to do)."""
    if capturing():
        _GRAVEYARD.append((None, obj))
        return True
    return False


def flush():
    """Free what was parked during captures this package did not open
    (torch.cuda.graph used directly: end_capture never runs for them).  Only at
    this explicit point -- never from an unrelated teardown -- because a graph
    captured outside the package may still replay kernels that use those
    buffers: call it once such graphs are gone.  No-op while any
    capture is open on the current stream."""
    if not capturing():
        _drain()


def begin_capture():
    _CAPTURE_DEPTH[0] += 1


def end_capture():
    """Leave a capture; after the outermost one, run the deferred releases."""
    _CAPTURE_DEPTH[0] = max(0, _CAPTURE_DEPTH[0] - 1)
    if _CAPTURE_DEPTH[0] == 0 and not capturing():
        _drain()


def graveyard_size():
    return len(_GRAVEYARD)
