"""utils.py surface of the reference (utils.py:49-162, variance_expension.pyx:8-111),
computed by the HIP kernels (numpy arrays in, numpy arrays out).

Unlike the reference (which reads ``config.L_MAX_SCALARS`` at call time,
utils.py:56), l_max is inferred from the array length.
"""
import math

import numpy as np

from . import _capi as C


def _dev(x):
    import torch
    if not torch.cuda.is_available():
        raise C.GibbsHipError("gibbssampler_amd.utils needs a ROCm GPU (no CPU fallback)")
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float64)).cuda()


def _lmax_of_real(n):
    L = int(round(math.sqrt(n))) - 1
    if (L + 1) ** 2 != n:
        raise ValueError("real a_lm array must have (L+1)^2 entries")
    return L


def _lmax_of_complex(n):
    L = int((-3 + math.sqrt(1 + 8 * n)) // 2)
    if (L + 1) * (L + 2) // 2 != n:
        raise ValueError("complex a_lm array must have (L+1)(L+2)/2 entries")
    return L


def generate_var_cl(cls_):
    """utils.generate_var_cl (utils.py:139-147): per-slot variance D_l 2pi/(l(l+1))."""
    lib = C.load()
    dl = np.atleast_2d(np.asarray(cls_, dtype=np.float64))
    L = dl.shape[-1] - 1
    import torch
    out = torch.zeros(dl.shape[0], (L + 1) ** 2, dtype=torch.float64, device="cuda")
    C.check(lib.gs_var_expand(L, dl.shape[0], C.ptr(_dev(dl)), C.ptr(out), C.stream_ptr()), "gs_var_expand")
    o = out.cpu().numpy()
    return o[0] if np.ndim(cls_) == 1 else o


generate_var_cl_cython = generate_var_cl


def real_to_complex(alms):
    """utils.real_to_complex (utils.py:49-60)."""
    lib = C.load()
    a = np.atleast_2d(np.asarray(alms, dtype=np.float64))
    L = _lmax_of_real(a.shape[-1])
    import torch
    out = torch.zeros(a.shape[0], (L + 1) * (L + 2), dtype=torch.float64, device="cuda")
    C.check(lib.gs_real_to_complex(L, a.shape[0], C.ptr(_dev(a)), C.ptr(out), C.stream_ptr()), "gs_real_to_complex")
    o = out.cpu().numpy().reshape(a.shape[0], -1, 2)
    c = o[..., 0] + 1j * o[..., 1]
    return c[0] if np.ndim(alms) == 1 else c


def complex_to_real(alms):
    """utils.complex_to_real (utils.py:63-76)."""
    lib = C.load()
    c = np.atleast_2d(np.asarray(alms, dtype=np.complex128))
    L = _lmax_of_complex(c.shape[-1])
    inter = np.stack([c.real, c.imag], axis=-1).reshape(c.shape[0], -1)
    import torch
    out = torch.zeros(c.shape[0], (L + 1) ** 2, dtype=torch.float64, device="cuda")
    C.check(lib.gs_complex_to_real(L, c.shape[0], C.ptr(_dev(inter)), C.ptr(out), C.stream_ptr()),
            "gs_complex_to_real")
    o = out.cpu().numpy()
    return o[0] if np.ndim(alms) == 1 else o


def remove_monopole_dipole_contributions(alms):
    """variance_expension.remove_monopole_dipole_contributions (variance_expension.pyx:103-111)."""
    lib = C.load()
    a = np.atleast_2d(np.asarray(alms, dtype=np.float64))
    L = _lmax_of_real(a.shape[-1])
    t = _dev(a)
    C.check(lib.gs_remove_monopole_dipole(L, a.shape[0], C.ptr(t), C.stream_ptr()), "gs_remove_monopole_dipole")
    o = t.cpu().numpy()
    return o[0] if np.ndim(alms) == 1 else o


def unfold_bins(binned_cls_, bins):
    """utils.unfold_bins (utils.py:150-162): host-side (setup-time) helper."""
    bins = np.asarray(bins)
    return np.repeat(np.asarray(binned_cls_, dtype=np.float64), bins[1:] - bins[:-1])


def alm2cl(alms, alms2=None):
    """hp.alm2cl on the real layout (CenteredGibbs.py:30,61)."""
    lib = C.load()
    a = np.atleast_2d(np.asarray(alms, dtype=np.float64))
    L = _lmax_of_real(a.shape[-1])
    b = a if alms2 is None else np.atleast_2d(np.asarray(alms2, dtype=np.float64))
    import torch
    out = torch.zeros(a.shape[0], L + 1, dtype=torch.float64, device="cuda")
    C.check(lib.gs_alm2cl(L, a.shape[0], C.ptr(_dev(a)), C.ptr(_dev(b)), C.ptr(out), C.stream_ptr()), "gs_alm2cl")
    o = out.cpu().numpy()
    return o[0] if np.ndim(alms) == 1 else o


def adjoint_synthesis_hp(map, bl_map=None, lmax=None):
    """utils.adjoint_synthesis_hp (utils.py:79-111) on the device SHT: the
    reference's "adjoint synthesis" Npix/(4 pi) * complex_to_real(map2alm(map,
    iter=3)) per field (healpy's default iter = 3, so like the reference this is
    the Jacobi-refined analysis, not the exact adjoint -- SURVEY.md Appendix
    B.9), times the real-layout beam diagonal ``bl_map`` when given.  One map
    (T) -> one array; three maps (T, Q, U) -> (alm_T, alm_E, alm_B).  ``lmax``
    defaults to 2 N_side, the reference's config.L_MAX_SCALARS."""
    import torch
    from .sht import HealpixSHT
    maps = np.asarray(map, dtype=np.float64)
    pol = maps.ndim == 2 and maps.shape[0] == 3
    npix = maps.shape[-1]
    nside = int(round(math.sqrt(npix / 12)))
    if 12 * nside * nside != npix:
        raise ValueError("map length is not 12 nside^2")
    L = 2 * nside if lmax is None else int(lmax)
    sht = HealpixSHT(nside, L)
    t = torch.from_numpy(np.ascontiguousarray(maps)).cuda()
    a = sht.map2alm(t, iter=3, layout="real", ncomp=3 if pol else 1).cpu().numpy() * (npix / (4 * math.pi))
    if bl_map is not None:
        a = a * np.asarray(bl_map, dtype=np.float64)
    return tuple(a) if pol else a
