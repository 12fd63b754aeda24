"""CPU restatement of the device synthetic-data path (gibbssampler_amd/data.py),
test infrastructure only: main_polarization.generate_dataset
(main_polarization.py:25-59) with healpy.synfast = synalm + smoothalm(pol=True)
+ alm2map, over the oracle SHT (oracle/sht.py), numpy legacy draws in the same
order (z for T, E, B; then pixel noise T, Q, U).  Parity unpinned against
healpy (absent); it pins the device arithmetic."""
import math

import numpy as np

from . import harmonic as H
from . import sht as O


def beams(L, fwhm_rad, F):
    sigma = fwhm_rad / math.sqrt(8.0 * math.log(2.0))
    ell = np.arange(L + 1, dtype=np.float64)
    g = np.exp(-0.5 * ell * (ell + 1) * sigma ** 2)
    gp = g * math.exp(2.0 * sigma ** 2)
    return {1: [g], 2: [gp, gp], 3: [g, gp, gp]}[F]


def synalm_real(rows, L, fwhm_rad, z):
    """rows: [TT] / [EE, BB] / [TT, EE, BB, TE] C_l; z [F, NR] -> real a_lm [F, NR]."""
    F = {1: 1, 2: 2, 4: 3}[len(rows)]
    sl = H.slot_ell(L)
    b = beams(L, fwhm_rad, F)
    if F == 3:
        tt, ee, bb, te = (np.asarray(r, dtype=np.float64)[:L + 1] for r in rows)
        a00 = np.sqrt(tt)
        a10 = np.where(tt != 0, te / np.where(tt != 0, a00, 1.0), 0.0)
        a11 = np.where(tt != 0, np.sqrt(np.maximum(ee - a10 ** 2, 0.0)), np.sqrt(ee))
        return np.stack([b[0][sl] * (a00[sl] * z[0]), b[1][sl] * (a10[sl] * z[0] + a11[sl] * z[1]),
                         b[2][sl] * (np.sqrt(bb)[sl] * z[2])])
    return np.stack([b[f][sl] * (np.sqrt(np.maximum(np.asarray(rows[f], dtype=np.float64)[:L + 1], 0.0))[sl]
                                 * z[f]) for f in range(F)])


def synfast(rows, nside, L, fwhm_rad, z):
    a = synalm_real(rows, L, fwhm_rad, z)
    nc = O._cidx(L)[0].shape[0]
    full = np.zeros((3, nc), dtype=np.complex128)
    if a.shape[0] == 1:
        full[0] = H.real_to_complex(a[0], L)
        return O.alm2map(full, nside, L)[0]
    for k, r in enumerate((1, 2) if a.shape[0] == 2 else (0, 1, 2)):
        full[r] = H.real_to_complex(a[k], L)
    m = O.alm2map(full, nside, L)
    return m if a.shape[0] == 3 else m[1:]


def generate_dataset(cls_, nside, L, fwhm_deg, var_noise_temp, var_noise_pol, polarization=True, mask=None,
                     reference_quirks=True):
    Npix = 12 * nside ** 2
    fwhm = math.radians(fwhm_deg)
    vt = np.broadcast_to(np.asarray(var_noise_temp, dtype=np.float64), (Npix,))
    vp = np.broadcast_to(np.asarray(var_noise_pol, dtype=np.float64), (Npix,))
    if polarization:
        rows = [np.asarray(cls_[k], dtype=np.float64) for k in range(4)]
        z = np.random.standard_normal((3, (L + 1) ** 2))
        truth = synfast(rows, nside, L, fwhm, z)
        d = truth.copy()
        d[0] += np.random.normal(scale=np.sqrt(vt))
        d[1] += np.random.normal(scale=np.sqrt(vp))
        d[2] += np.random.normal(scale=np.sqrt(vp))
        map_true = d if reference_quirks else truth
        if mask is None:
            a = O.map2alm(d, nside, L, iter=3)
            return map_true, {"EE": H.complex_to_real(a[1], L), "BB": H.complex_to_real(a[2], L)}, \
                {"Q": d[1], "U": d[2]}
        return map_true, {"Q": d[1] * mask, "U": d[2] * mask}
    cl = np.atleast_2d(np.asarray(cls_, dtype=np.float64))[0]
    z = np.random.standard_normal((1, (L + 1) ** 2))
    truth = synfast([cl], nside, L, fwhm, z)
    d = truth + np.random.normal(scale=np.sqrt(vt))
    map_true = d if reference_quirks else truth
    return None, cls_, map_true, (d if mask is None else d * mask)
