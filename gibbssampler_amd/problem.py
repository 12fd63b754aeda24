"""Synthetic full-sky problems -- the harmonic-space analogue of
main_polarization.generate_dataset (main_polarization.py:25-59) for the
all_sph / full-sky configuration, plus the reference's binning, MH blocking
and proposal-variance recipes (config.py:45-55, 119-132, 192-197).

classy is unavailable offline, so spectra are the analytic fiducial
D^TT = 1000, D^EE = 10 (l/100)^0.5, D^BB = 0.01, D^TE = 0.5 sqrt(TT EE)
(muK^2, zero below l = 2).
"""
import math

import numpy as np

SPECTRA = {1: ("TT",), 2: ("EE", "BB"), 3: ("TT", "EE", "BB", "TE")}
FIELDS = {1: ("TT",), 2: ("EE", "BB"), 3: ("TT", "EE", "BB")}

# config.py:45 -- Planck BB bins, hard-wired to L = 512
BINS_BB_512 = np.concatenate([np.arange(0, 396),
                              np.array([396, 398, 400, 402, 406, 410, 415, 420, 425, 430, 435, 440, 445,
                                        460, 475, 495, 513])])


def gauss_beam(fwhm_rad, lmax):
    """healpy.gauss_beam semantics (GibbsSampler.py:72): exp(-l(l+1) sigma^2/2)."""
    sigma = fwhm_rad / math.sqrt(8.0 * math.log(2.0))
    ell = np.arange(lmax + 1, dtype=np.float64)
    return np.exp(-0.5 * ell * (ell + 1) * sigma ** 2)


def slot_ell(lmax):
    """multipole of each real-layout slot (utils.py:49-76)."""
    L = lmax
    out = [np.arange(L + 1)]
    for m in range(1, L + 1):
        out.append(np.repeat(np.arange(m, L + 1), 2))
    return np.concatenate(out)


def fiducial_dl(lmax, nfields):
    ell = np.arange(lmax + 1, dtype=np.float64)
    on = ell >= 2
    tt = np.where(on, 1000.0, 0.0)
    ee = np.where(on, 10.0 * (np.maximum(ell, 1) / 100.0) ** 0.5, 0.0)
    bb = np.where(on, 0.01, 0.0)
    te = 0.5 * np.sqrt(tt * ee)
    full = {"TT": tt, "EE": ee, "BB": bb, "TE": te}
    return {s: full[s] for s in SPECTRA[nfields]}


def default_bins(lmax, nfields):
    """EE/TT/TE unbinned (config.py:46); BB = Planck bins at L = 512, else unbinned."""
    bins = {}
    for s in SPECTRA[nfields]:
        if s == "BB" and lmax == 512:
            bins[s] = BINS_BB_512.copy()
        else:
            bins[s] = np.arange(0, lmax + 2)
    return bins


def default_blocks(lmax, bins):
    """config.py:51-55: one block for EE (and TT, TE); BB = [2, 279] + one block per
    bin above it at L = 512, generalised to [2, floor(0.545 L)] + per-bin."""
    blocks = {}
    for s, b in bins.items():
        nb = len(b) - 1
        if s == "BB":
            k = 279 if lmax == 512 else int(0.545 * lmax)
            k = min(max(k, 3), nb)
            blocks[s] = np.concatenate([[2, k], np.arange(k + 1, nb + 1)])
        else:
            blocks[s] = np.array([2, nb + 1])
    return blocks


def proposal_variances(lmax, nside, bins, bl, noise_var_pol, noise_var_temp=None, fsky=1.0):
    """config.py:119-132 (binned_variances_pol) with the preliminary-run choice
    proposal = binned[2:] (config.py:192-197); TT uses the temperature noise,
    TE the geometric mean."""
    Npix = 12 * nside ** 2
    w = 4 * np.pi / Npix
    ell = np.arange(lmax + 1, dtype=np.float64)
    scale = (ell * (ell + 1)) ** 2 * 2 / (4 * np.pi ** 2 * (2 * ell + 1))
    out = {}
    for s, b in bins.items():
        if s == "TT":
            nv = noise_var_temp
        elif s == "TE":
            nv = math.sqrt(noise_var_temp * noise_var_pol)
        else:
            nv = noise_var_pol
        unb = (w * nv / bl ** 2) ** 2 * scale / fsky
        binned = np.array([np.mean(unb[b[i]:b[i + 1]]) / (b[i + 1] - b[i]) for i in range(len(b) - 1)])
        out[s] = binned[2:]
    return out


def bin_spectrum(dl, b):
    """main_polarization.py:140-146: mean of D_l over each bin."""
    return np.array([np.mean(dl[b[i]:b[i + 1]]) for i in range(len(b) - 1)])


def synthetic_problem(lmax, nside, nfields, seed=0, fwhm_deg=0.5, noise_var_temp=40.0 ** 2,
                      noise_var_pol=0.2 ** 2, bins=None, blocks=None):
    """d = b s_true + n in the real harmonic layout, s_true ~ N(0, C_l)."""
    L = int(lmax)
    rng = np.random.RandomState(seed)
    spectra = SPECTRA[nfields]
    bl = gauss_beam(fwhm_deg * np.pi / 180.0, L)
    noise = {1: [noise_var_temp], 2: [noise_var_pol] * 2, 3: [noise_var_temp, noise_var_pol, noise_var_pol]}[nfields]
    dl = fiducial_dl(L, nfields)
    ell = np.arange(L + 1, dtype=np.float64)
    fac = np.zeros(L + 1)
    fac[1:] = 2 * np.pi / (ell[1:] * (ell[1:] + 1))
    sl = slot_ell(L)
    NR = (L + 1) ** 2
    z = rng.normal(size=(nfields, NR))
    if nfields == 3:
        tt, ee, te, bb = (dl[s] * fac for s in ("TT", "EE", "TE", "BB"))
        a00 = np.sqrt(tt)
        a10 = np.where(a00 > 0, te / np.where(a00 > 0, a00, 1), 0.0)
        a11 = np.sqrt(np.maximum(ee - a10 ** 2, 0.0))
        s_true = np.stack([a00[sl] * z[0], a10[sl] * z[0] + a11[sl] * z[1], np.sqrt(bb)[sl] * z[2]])
    else:
        s_true = np.stack([np.sqrt(dl[s] * fac)[sl] * z[k] for k, s in enumerate(spectra)])
    Npix = 12 * nside ** 2
    kappa = np.array([Npix / (4 * np.pi * v) for v in noise])
    d = bl[sl] * s_true + rng.normal(size=(nfields, NR)) / np.sqrt(kappa)[:, None]
    bins = default_bins(L, nfields) if bins is None else bins
    blocks = default_blocks(L, bins) if blocks is None else blocks
    pv = proposal_variances(L, nside, bins, bl, noise_var_pol, noise_var_temp)
    init = {s: bin_spectrum(dl[s], bins[s]) for s in spectra}
    return dict(lmax=L, nside=nside, nfields=nfields, bl=bl, noise_var=np.array(noise, dtype=np.float64),
                bins=bins, blocks=blocks, proposal_variances=pv, d_alm=d, dls_init=init, dl_true=dl)
