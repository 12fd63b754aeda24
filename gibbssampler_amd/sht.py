"""HEALPix RING spherical-harmonic transforms on the GPU (libgibbs_hip.so).

Device replacement for the healpy calls of the reference's masked paths:
``hp.alm2map`` (CenteredGibbs.py:204,505,698,751,791; NonCenteredGibbs.py:350),
``hp.map2alm`` (``iter=0`` at CenteredGibbs.py:298,513,717,773,812; default
``iter=3`` at utils.py:89,104 and NonCenteredGibbs.py:155) and
``utils.adjoint_synthesis_hp`` (utils.py:79-111).  Conventions: oracle/sht.py
(HEALPix / Zaldarriaga-Seljak).

All arrays are torch float64 tensors on the current CUDA (HIP) device.  a_lm
are in the build's real m-major layout (``layout="real"``, (L+1)^2 per
component, utils.py:49-76) or healpy's complex order (``layout="complex"``:
complex128 tensors of (L+1)(L+2)/2 per component).
"""
import ctypes

import torch

from . import _capi

_LAYOUT = {"real": _capi.GS_ALM_REAL, "complex": _capi.GS_ALM_COMPLEX}


class HealpixSHT:
    """One device SHT plan for (nside, lmax): ring geometry, recurrence
    coefficients, Legendre start tables and ring-FFT kernels built once."""

    def __init__(self, nside, lmax):
        self.lib = _capi.load()
        self.nside, self.lmax = int(nside), int(lmax)
        self.npix = 12 * self.nside ** 2
        h = ctypes.c_void_p()
        _capi.check(self.lib.gs_sht_create(self.nside, self.lmax, ctypes.byref(h)), "gs_sht_create")
        self.handle = h
        nb = ctypes.c_longlong()
        _capi.check(self.lib.gs_sht_info(h, None, None, None, ctypes.byref(nb)), "gs_sht_info")
        self.device_bytes = nb.value

    def __del__(self):
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            _capi.release(self.lib.gs_sht_destroy, h)
            self.handle = None

    def set_mfma(self, on=True):
        """Route the Legendre stage through the fp64 matrix cores (plan-time
        lambda / F1 / F2 table; small maps; gs_sht_set_mfma)."""
        _capi.check(self.lib.gs_sht_set_mfma(self.handle, int(bool(on))), "gs_sht_set_mfma")
        return self

    @property
    def mfma(self):
        on, nb = ctypes.c_int(), ctypes.c_longlong()
        _capi.check(self.lib.gs_sht_mfma_info(self.handle, ctypes.byref(on), ctypes.byref(nb)), "gs_sht_mfma_info")
        return bool(on.value), nb.value

    def alm2map_batch(self, alm, ncomp, bl=None, layout="real", out=None):
        """alm [B, ncomp, n] -> maps [B, ncomp, Npix] in one batched transform
        (optionally the per-l beam on the input load, real layout)."""
        B = alm.shape[0]
        a = alm.contiguous()
        if layout == "complex":
            a = torch.view_as_real(a)
        if out is None:
            out = torch.empty((B, ncomp, self.npix), dtype=torch.float64, device=alm.device)
        _capi.check(self.lib.gs_sht_alm2map_batch(self.handle, B, ncomp, _LAYOUT[layout], _capi.ptr(a),
                                                  _capi.ptr(None if bl is None else bl.contiguous()), _capi.ptr(out),
                                                  _capi.stream_ptr()), "gs_sht_alm2map_batch")
        return out

    def map2alm_batch(self, maps, ncomp, iter=0, weights=None, layout="real", out=None):
        """maps [B, ncomp, Npix] -> alm [B, ncomp, n] in one batched transform
        (optionally of weights * maps, weights [ncomp, Npix] shared by the batch)."""
        B = maps.shape[0]
        maps = maps.contiguous()
        if out is None:
            if layout == "complex":
                out = torch.empty((B, ncomp, self.ncomplex), dtype=torch.complex128, device=maps.device)
            else:
                out = torch.empty((B, ncomp, self.nreal), dtype=torch.float64, device=maps.device)
        o = torch.view_as_real(out) if layout == "complex" else out
        _capi.check(self.lib.gs_sht_map2alm_batch(self.handle, B, ncomp, _LAYOUT[layout], _capi.ptr(maps),
                                                  _capi.ptr(None if weights is None else weights.contiguous()),
                                                  _capi.ptr(o), int(iter), _capi.stream_ptr()), "gs_sht_map2alm_batch")
        return out

    def apply_weighted_batch(self, alm, ncomp, weights, bl=None, out=None):
        """alm [B, ncomp, n] (real layout) -> map2alm(weights * alm2map(bl x alm)):
        the masked PCG operator's transform pair (CenteredGibbs.py:448-491), the
        maps kept on chip on the table path (gs_sht_apply_weighted_batch)."""
        B = alm.shape[0]
        a = alm.contiguous()
        w = weights.contiguous()
        if out is None:
            out = torch.empty((B, ncomp, self.nreal), dtype=torch.float64, device=alm.device)
        scratch = torch.empty((B, ncomp, self.npix), dtype=torch.float64, device=alm.device)
        _capi.check(self.lib.gs_sht_apply_weighted_batch(self.handle, B, ncomp, _capi.ptr(a),
                                                         _capi.ptr(None if bl is None else bl.contiguous()),
                                                         _capi.ptr(w), _capi.ptr(scratch), _capi.ptr(out),
                                                         _capi.stream_ptr()), "gs_sht_apply_weighted_batch")
        return out

    # -- shapes -----------------------------------------------------------------
    @property
    def nreal(self):
        return (self.lmax + 1) ** 2

    @property
    def ncomplex(self):
        return (self.lmax + 1) * (self.lmax + 2) // 2

    def _alm_view(self, alm, layout, ncomp):
        if layout == "complex":
            if alm.dtype != torch.complex128:
                raise TypeError("complex layout needs complex128 a_lm")
            alm = alm.contiguous()
            if alm.numel() != ncomp * self.ncomplex:
                raise ValueError("a_lm size does not match (ncomp, lmax)")
            return torch.view_as_real(alm)
        if alm.dtype != torch.float64:
            raise TypeError("real layout needs float64 a_lm")
        alm = alm.contiguous()
        if alm.numel() != ncomp * self.nreal:
            raise ValueError("a_lm size does not match (ncomp, lmax)")
        return alm

    # -- transforms -----------------------------------------------------------------
    def alm2map(self, alm, ncomp=None, layout="real", out=None):
        """alm [ncomp, n] -> maps [ncomp, Npix].  ncomp 1: T; 2: (E,B)->(Q,U);
        3: (T,E,B)->(T,Q,U)."""
        if ncomp is None:
            ncomp = 1 if alm.dim() == 1 else alm.shape[0]
        a = self._alm_view(alm, layout, ncomp)
        if out is None:
            out = torch.empty((ncomp, self.npix) if ncomp > 1 else (self.npix,), dtype=torch.float64,
                              device=alm.device)
        _capi.check(self.lib.gs_sht_alm2map(self.handle, ncomp, _LAYOUT[layout], _capi.ptr(a), _capi.ptr(out),
                                            _capi.stream_ptr()), "gs_sht_alm2map")
        return out

    def map2alm(self, maps, iter=0, layout="real", ncomp=None, out=None):
        """maps [ncomp, Npix] -> alm; (4pi/Npix) x adjoint, plus ``iter`` Jacobi steps."""
        if ncomp is None:
            ncomp = 1 if maps.dim() == 1 else maps.shape[0]
        maps = maps.contiguous()
        if maps.dtype != torch.float64 or maps.numel() != ncomp * self.npix:
            raise ValueError("maps must be float64 [ncomp, 12 nside^2]")
        if out is None:
            if layout == "complex":
                out = torch.empty((ncomp, self.ncomplex) if ncomp > 1 else (self.ncomplex,), dtype=torch.complex128,
                                  device=maps.device)
            else:
                out = torch.empty((ncomp, self.nreal) if ncomp > 1 else (self.nreal,), dtype=torch.float64,
                                  device=maps.device)
        o = torch.view_as_real(out) if layout == "complex" else out
        _capi.check(self.lib.gs_sht_map2alm(self.handle, ncomp, _LAYOUT[layout], _capi.ptr(maps), _capi.ptr(o),
                                            int(iter), _capi.stream_ptr()), "gs_sht_map2alm")
        return out

    def alm2map_beamed(self, alm, bl, ncomp=None, out=None):
        """alm2map of b_l * alm (real layout) with the beam applied on the input
        load: hp.alm2map(almxfl(alm, bl)) of CenteredGibbs.py:698-699."""
        if ncomp is None:
            ncomp = 1 if alm.dim() == 1 else alm.shape[0]
        a = self._alm_view(alm, "real", ncomp)
        bl = bl.contiguous()
        if bl.dtype != torch.float64 or bl.numel() < self.lmax + 1:
            raise ValueError("bl must be float64 [lmax + 1]")
        if out is None:
            out = torch.empty((ncomp, self.npix) if ncomp > 1 else (self.npix,), dtype=torch.float64,
                              device=alm.device)
        _capi.check(self.lib.gs_sht_alm2map_beamed(self.handle, ncomp, _capi.ptr(a), _capi.ptr(bl), _capi.ptr(out),
                                                   _capi.stream_ptr()), "gs_sht_alm2map_beamed")
        return out

    def map2alm_weighted(self, maps, weights, ncomp=None, out=None):
        """map2alm(weights * maps, iter=0) into the real layout, the product formed
        on the ring stage's input load (CenteredGibbs.py:298-299,510-513)."""
        if ncomp is None:
            ncomp = 1 if maps.dim() == 1 else maps.shape[0]
        maps, weights = maps.contiguous(), weights.contiguous()
        for t in (maps, weights):
            if t.dtype != torch.float64 or t.numel() != ncomp * self.npix:
                raise ValueError("maps / weights must be float64 [ncomp, 12 nside^2]")
        if out is None:
            out = torch.empty((ncomp, self.nreal) if ncomp > 1 else (self.nreal,), dtype=torch.float64,
                              device=maps.device)
        _capi.check(self.lib.gs_sht_map2alm_weighted(self.handle, ncomp, _capi.ptr(maps), _capi.ptr(weights),
                                                     _capi.ptr(out), _capi.stream_ptr()), "gs_sht_map2alm_weighted")
        return out

    def adjoint_synthesis(self, maps, bl=None, iter=3):
        """utils.adjoint_synthesis_hp (utils.py:79-111): map2alm(iter) rescaled by
        Npix/(4pi), real layout, optionally times the per-slot beam ``bl``
        (a length-(L+1)^2 tensor, or per-l of length L+1)."""
        a = self.map2alm(maps, iter=iter, layout="real")
        a = a * (self.npix / (4.0 * torch.pi))
        if bl is not None:
            if bl.numel() == self.lmax + 1:
                from .problem import slot_ell
                idx = torch.as_tensor(slot_ell(self.lmax), device=a.device)
                bl = bl.to(a.device)[idx]
            a = a * bl
        return a
