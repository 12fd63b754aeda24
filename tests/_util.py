"""Shared helpers for the parity tests: oracle <-> device layouts."""
import numpy as np

from oracle import harmonic as H


def stats_rows(F, st):
    """oracle sweep_stats dict -> [nstat, L+1] rows of include/gibbs_capi.h."""
    ss, ds = st["ss"], st["ds"]
    if F == 1:
        return np.stack([ss[0, 0], ds[0, 0]])
    if F == 2:
        return np.stack([ss[0, 0], ss[1, 1], ds[0, 0], ds[1, 1]])
    return np.stack([ss[0, 0], ss[1, 1], ss[2, 2], ss[0, 1], ds[0, 0], ds[1, 0], ds[1, 1], ds[2, 2]])


def rows_to_stats(F, r):
    """[nstat, L+1] device rows -> oracle stats dict (symmetric ss, lower ds)."""
    Lp1 = r.shape[-1]
    ss = np.zeros((F, F, Lp1))
    ds = np.zeros((F, F, Lp1))
    if F == 1:
        ss[0, 0], ds[0, 0] = r[0], r[1]
    elif F == 2:
        ss[0, 0], ss[1, 1], ds[0, 0], ds[1, 1] = r[0], r[1], r[2], r[3]
    else:
        ss[0, 0], ss[1, 1], ss[2, 2] = r[0], r[1], r[2]
        ss[0, 1] = ss[1, 0] = r[3]
        ds[0, 0], ds[1, 0], ds[1, 1], ds[2, 2] = r[4], r[5], r[6], r[7]
    return {"ss": ss, "ds": ds}


def fiducial_dl(L, F):
    """SURVEY.md 8d analytic fiducial (muK^2), zero for l < 2."""
    ell = np.arange(L + 1, dtype=np.float64)
    on = ell >= 2
    tt = np.where(on, 1000.0, 0.0)
    ee = np.where(on, 10.0 * (np.maximum(ell, 1) / 100.0) ** 0.5, 0.0)
    bb = np.where(on, 0.01, 0.0)
    te = 0.5 * np.sqrt(tt * ee)
    if F == 1:
        return {"TT": tt}
    if F == 2:
        return {"EE": ee, "BB": bb}
    return {"TT": tt, "EE": ee, "BB": bb, "TE": te}


def make_problem(L, nside, F, seed=0, binned_bb=True, fwhm_deg=None):
    """Synthetic full-sky problem: d = b s_true + n in the real harmonic layout."""
    rng = np.random.RandomState(seed)
    Npix = 12 * nside ** 2
    fwhm = (fwhm_deg if fwhm_deg is not None else max(0.5, 180.0 / L * 2)) * np.pi / 180
    bl = H.gauss_beam(fwhm, L)
    noise = {1: [40.0 ** 2], 2: [0.2 ** 2] * 2, 3: [40.0 ** 2, 0.2 ** 2, 0.2 ** 2]}[F]
    spectra = H.SPECTRA[F]
    dl = fiducial_dl(L, F)
    ell = H.slot_ell(L)
    var = {s: H.var_from_dl(dl[s]) for s in spectra}
    kap = [12 * nside ** 2 / (4 * np.pi * v) for v in noise]
    zs = rng.normal(size=(F, (L + 1) ** 2))
    if F == 3:
        C = H.cov_blocks(H.Model(L, nside, 3, bl, noise, {s: np.arange(L + 2) for s in spectra}),
                         np.stack([dl[s] for s in spectra]))
        A = np.zeros_like(C)
        for l in range(L + 1):
            w, V = np.linalg.eigh(C[l])
            A[l] = V @ np.diag(np.sqrt(np.maximum(w, 0)))
        s_true = np.einsum("sfg,gs->fs", A[ell], zs)
    else:
        s_true = np.stack([np.sqrt(var[s])[ell] * zs[k] for k, s in enumerate(spectra)])
    d = bl[ell] * s_true + rng.normal(size=(F, (L + 1) ** 2)) / np.sqrt(np.array(kap))[:, None]
    bins = {}
    for s in spectra:
        if s == "BB" and binned_bb:
            cut = (2 * L) // 3
            b = np.concatenate([np.arange(0, cut), np.arange(cut, L + 1, 5), [L + 1]])
            bins[s] = np.unique(b)
        else:
            bins[s] = np.arange(0, L + 2)
    blocks = {}
    for s in spectra:
        nb = len(bins[s]) - 1
        if s == "BB" and binned_bb:
            k = max(3, (nb * 2) // 3)
            blocks[s] = np.concatenate([[2, k], np.arange(k + 1, nb + 1)])
        else:
            blocks[s] = np.array([2, nb + 1])
    w = 4 * np.pi / Npix
    lv = np.arange(L + 1, dtype=np.float64)
    scale = (lv * (lv + 1)) ** 2 * 2 / (4 * np.pi ** 2 * (2 * lv + 1))
    pv = {}
    for k, s in enumerate(spectra):
        nv = noise[min(k, F - 1)] if F != 3 else {"TT": noise[0], "EE": noise[1], "BB": noise[2], "TE": np.sqrt(noise[0] * noise[1])}[s]
        unb = (w * nv / bl ** 2) ** 2 * scale
        b = bins[s]
        binned = np.array([np.mean(unb[b[i]:b[i + 1]]) / (b[i + 1] - b[i]) for i in range(len(b) - 1)])
        pv[s] = binned[2:]
    init = {s: np.array([np.mean(dl[s][bins[s][i]:bins[s][i + 1]]) for i in range(len(bins[s]) - 1)])
            for s in spectra}
    model = H.Model(L=L, nside=nside, nfields=F, bl=bl, noise_var=noise, bins=bins, blocks=blocks,
                    proposal_variances=pv, d_alm=d)
    return model, init
