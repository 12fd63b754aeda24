"""Synthetic observations on the device: the
``generate_dataset`` of main_polarization.py:25-59 with healpy.synfast
(synalm + Gaussian smoothing + alm2map) restated over the build's kernels:

  a_lm = b_l C_l^1/2 z          gs_synalm (per real slot; TEB via the (T, E)
                                 Cholesky factor, healpy's new=True order
                                 TT, EE, BB, TE)
  map  = alm2map(a_lm)          gs_sht (HEALPix RING, spin 0 and spin 2)
  d    = map + sigma n          per pixel (np.random.normal order T, Q, U)
  E, B = map2alm(d, iter=3)     full-sky harmonic data (main_polarization.py:44)

The beam follows healpy.smoothalm(pol=True): b_l = exp(-l(l+1) sigma^2 / 2)
for T and b_l exp(2 sigma^2) for E, B.  Draws come from numpy's legacy
global stream (z for T, E, B then the pixel noise), so a seeded run is
reproducible; healpy's own synalm draw order is not restated (healpy is
absent: parity of the draws with healpy is unpinned, the arithmetic is
checked against oracle/ at small sizes).
"""
import math

import numpy as np
import torch

from . import _capi
from .sht import HealpixSHT


def pixel_cos_theta(nside):
    """cos(theta) of every HEALPix RING pixel (Gorski et al. 2005 ring latitudes)."""
    N = int(nside)
    i = np.arange(1, 4 * N, dtype=np.float64)
    z = np.where(i < N, 1.0 - i * i / (3.0 * N * N),
                 np.where(i <= 3 * N, 4.0 / 3.0 - 2.0 * i / (3.0 * N), -(1.0 - (4 * N - i) ** 2 / (3.0 * N * N))))
    ii = np.arange(1, 4 * N, dtype=np.int64)
    nphi = np.where(ii < N, 4 * ii, np.where(ii <= 3 * N, 4 * N, 4 * (4 * N - ii)))
    return np.repeat(z, nphi)


def band_mask(nside, cut=0.2):
    """the synthetic 80% mask of SURVEY.md 8d: keep |cos theta| > cut."""
    return (np.abs(pixel_cos_theta(nside)) > cut).astype(np.float64)


def pixel_phi(nside):
    """phi of every HEALPix RING pixel (healpy pix2ang: polar ring i at (j + 1/2)
    pi / (2 i), equatorial ring i at (j + 1/2 [i + N even]) pi / (2 N))."""
    N = int(nside)
    out = []
    for i in range(1, 4 * N):
        ip = i if i < N else (4 * N - i if i > 3 * N else N)
        n = 4 * ip
        j = np.arange(n, dtype=np.float64)
        if i < N or i > 3 * N:
            out.append((j + 0.5) * np.pi / (2 * ip))
        else:
            out.append((j + (0.5 if (i + N) % 2 == 0 else 0.0)) * np.pi / (2 * N))
    return np.concatenate(out)


def galactic_mask(nside, cut=0.2, wave=(0.12, 0.06)):
    """a galactic-plane-like 80% mask whose edge is not a ring: keep |cos theta| >
    cut + wave[0] sin(2 phi) + wave[1] cos(3 phi + 1) (f_sky 0.8 on average).  A
    galactic cut in galactic coordinates leaves the polar caps whole and cuts
    the rings near the plane along a wavy edge: the rings that cross it have
    varying weights, the others a constant one (the ring classes of
    gs_sht_register_weights) -- the realistic counterpart of band_mask, whose
    every ring is whole or cut."""
    z, ph = pixel_cos_theta(nside), pixel_phi(nside)
    edge = cut + wave[0] * np.sin(2.0 * ph) + wave[1] * np.cos(3.0 * ph + 1.0)
    return (np.abs(z) > edge).astype(np.float64)


def _beams(lmax, fwhm_rad, nfields):
    sigma = fwhm_rad / math.sqrt(8.0 * math.log(2.0))
    ell = np.arange(lmax + 1, dtype=np.float64)
    g = np.exp(-0.5 * ell * (ell + 1) * sigma ** 2)
    gp = g * math.exp(2.0 * sigma ** 2)
    return {1: [g], 2: [gp, gp], 3: [g, gp, gp]}[nfields]


def synalm(cls_, lmax, fwhm_rad=0.0, z=None, device="cuda"):
    """real-layout a_lm [F, (L+1)^2] of a Gaussian sky with spectra ``cls_``
    (C_l; 1 row TT, or 4 rows TT, EE, BB, TE -> T, E, B; a dict with "EE",
    "BB" -> E, B), smoothed by the Gaussian beam."""
    L = int(lmax)
    NR = (L + 1) ** 2
    if isinstance(cls_, dict):
        rows = [np.asarray(cls_[s], dtype=np.float64)[:L + 1] for s in ("EE", "BB")]
        F = 2
    else:
        c = np.atleast_2d(np.asarray(cls_, dtype=np.float64))
        if c.shape[0] == 1:
            rows, F = [c[0, :L + 1]], 1
        elif c.shape[0] >= 4:
            rows, F = [c[k, :L + 1] for k in range(4)], 3
        else:
            raise ValueError("cls_ must have 1 (TT) or 4 (TT, EE, BB, TE) rows")
    if any(len(r) < L + 1 for r in rows):
        raise ValueError("cls_ shorter than lmax + 1")
    if z is None:
        z = np.random.standard_normal((F, NR))
    zt = torch.as_tensor(np.ascontiguousarray(z, dtype=np.float64).reshape(F, NR), device=device)
    cl = torch.as_tensor(np.ascontiguousarray(np.stack(rows)), device=device)
    beam = torch.as_tensor(np.ascontiguousarray(np.stack(_beams(L, fwhm_rad, F))), device=device)
    alm = torch.empty((F, NR), dtype=torch.float64, device=device)
    lib = _capi.load()
    _capi.check(lib.gs_synalm(L, F, _capi.ptr(cl), _capi.ptr(beam), _capi.ptr(zt), _capi.ptr(alm),
                              _capi.stream_ptr()), "gs_synalm")
    return alm


def synfast(cls_, nside, lmax, fwhm_rad=0.0, z=None, device="cuda"):
    """healpy.synfast(cls_, nside, lmax, fwhm, new=True): maps [3, Npix]
    (T, Q, U) for 4-row spectra, [Npix] for TT; device tensor."""
    alm = synalm(cls_, lmax, fwhm_rad, z, device)
    sht = HealpixSHT(nside, lmax)
    if alm.shape[0] == 1:
        return sht.alm2map(alm[0], ncomp=1)
    if alm.shape[0] == 2:
        return sht.alm2map(alm, ncomp=2)
    return sht.alm2map(alm, ncomp=3)


def generate_dataset(cls_, nside, lmax, fwhm_deg=0.5, var_noise_temp=40.0 ** 2, var_noise_pol=0.2 ** 2,
                     polarization=True, mask=None, reference_quirks=True, device="cuda"):
    """main_polarization.generate_dataset (main_polarization.py:25-59).

    polarization, no mask -> (map_true, {"EE", "BB": real-layout map2alm(d,
    iter=3)}, {"Q", "U"}); with a mask -> (map_true, {"Q": Q mask, "U": U mask});
    temperature -> (None, cls_, map_true, d[*mask]) (the reference returns an
    undefined ``theta_`` there).  ``reference_quirks``: the reference adds
    the noise to ``d = map_true`` in place, so its ``map_true`` carries the
    noise; set False for the noiseless sky.  Arrays are numpy (host)."""
    L = int(lmax)
    Npix = 12 * int(nside) ** 2
    fwhm = math.radians(fwhm_deg)
    vt = np.broadcast_to(np.asarray(var_noise_temp, dtype=np.float64), (Npix,))
    vp = np.broadcast_to(np.asarray(var_noise_pol, dtype=np.float64), (Npix,))
    m = None if mask is None else np.asarray(mask, dtype=np.float64)
    if polarization:
        maps = synfast(cls_, nside, L, fwhm, device=device)
        truth = maps.cpu().numpy()
        d = truth.copy()
        d[0] += np.random.normal(scale=np.sqrt(vt))
        d[1] += np.random.normal(scale=np.sqrt(vp))
        d[2] += np.random.normal(scale=np.sqrt(vp))
        map_true = d if reference_quirks else truth
        if m is None:
            sht = HealpixSHT(nside, L)
            alm = sht.map2alm(torch.as_tensor(d, device=device), iter=3, ncomp=3).cpu().numpy()
            return map_true, {"EE": alm[1], "BB": alm[2]}, {"Q": d[1], "U": d[2]}
        return map_true, {"Q": d[1] * m, "U": d[2] * m}
    cl = np.atleast_2d(np.asarray(cls_, dtype=np.float64))[0]
    truth = synfast(cl[None], nside, L, fwhm, device=device).cpu().numpy()
    d = truth + np.random.normal(scale=np.sqrt(vt))
    map_true = d if reference_quirks else truth
    return None, cls_, map_true, (d if m is None else d * m)
