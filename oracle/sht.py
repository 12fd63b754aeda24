"""numpy restatement of the HEALPix RING spherical-harmonic transforms (TEST INFRASTRUCTURE).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import
this module; the product path never does.

What it restates.  The reference never implements an SHT itself: it calls
healpy (``hp.alm2map`` at CenteredGibbs.py:204,505,698,751,791 and
NonCenteredGibbs.py:350; ``hp.map2alm`` with ``iter=0`` at
CenteredGibbs.py:298,513,717,773,812 and the default ``iter=3`` at
utils.py:89,104 and NonCenteredGibbs.py:155).  healpy (libsharp / ducc0, C++)
is absent offline and no reference test pins an SHT output, so this oracle is
**parity unpinned** against healpy: it follows the published HEALPix
conventions (Gorski et al. 2005; Zaldarriaga & Seljak 1997 for spin 2,
SURVEY.md Appendix A.4) and is itself pinned by analytic known answers
(closed-form Y_lm and +-2Y_lm, scipy.special.sph_harm_y, adjointness,
Parseval, band-limited round trips) in tests/test_oracle_sht.py.

Conventions.
  * RING pixelisation: north cap ring i = 1..N-1 has z = 1 - i^2/(3N^2),
    4i pixels at phi_j = (j + 1/2) pi / (2i); equatorial rings
    i = N..3N have z = 4/3 - 2i/(3N), 4N pixels at
    phi_j = (j + (1 - (i - N) mod 2)/2) pi / (2N); the south cap mirrors the
    north.  Pixels are numbered ring by ring from the north pole.
  * lambda_lm(x) = sqrt((2l+1)/(4pi) (l-m)!/(l+m)!) P_l^m(x) with the
    Condon-Shortley phase, Y_lm = lambda_lm e^{i m phi}.
  * spin 2: +-2Y_lm = (F1_lm +- F2_lm) e^{i m phi} with
        F1 = c_l [ -((l - m^2)/(1-x^2) + l(l-1)/2) lambda_lm + f_lm x/(1-x^2) lambda_{l-1,m} ]
        F2 = c_l m/(1-x^2) [ -(l-1) x lambda_lm + f_lm lambda_{l-1,m} ]
    c_l = 2/sqrt((l-1)l(l+1)(l+2)), f_lm = sqrt((2l+1)/(2l-1) (l^2-m^2));
    Q + iU = -sum (a_E + i a_B) 2Y_lm  (HEALPix / COSMO sign).
  * alm2map:  T = sum_m c_m Re[sum_l a_T lambda e^{im phi}], c_0 = 1, c_m = 2,
              Q = -sum_m c_m Re[sum_l (a_E F1 + i a_B F2) e^{im phi}],
              U = -sum_m c_m Re[sum_l (a_B F1 - i a_E F2) e^{im phi}].
  * map2alm(iter=0) = (4pi/Npix) x the exact adjoint of alm2map on the complex
    coefficients (healpy with uniform weights):
              a_T = w sum_p T lambda e^{-im phi},
              a_E = -w sum_p (Q F1 + i U F2) e^{-im phi},
              a_B = -w sum_p (U F1 - i Q F2) e^{-im phi};
    map2alm(iter=n) adds n Jacobi steps a += map2alm(m - alm2map(a)).
  * complex coefficients use healpy's m-major order idx = m(2L+1-m)/2 + l.

The ring sums are evaluated directly (no FFT), so this oracle shares neither
the FFT, the aliasing fold nor the scaled Legendre recurrence of the device
code.  Sizes: intended for N_side <= 64, l_max <= 128 (dense [ring, l, m]
tables; the unscaled recurrence is asserted not to underflow).
"""
import functools
import math

import numpy as np

FOURPI = 4.0 * math.pi


# ----------------------------------------------------------------------------
# geometry
# ----------------------------------------------------------------------------
def npix(nside):
    return 12 * nside * nside


def ring_info(nside):
    """Per ring (4N-1 of them, north to south): z = cos(theta), nphi, phi0,
    first pixel index."""
    N = nside
    nr = 4 * N - 1
    z = np.empty(nr)
    nphi = np.empty(nr, dtype=np.int64)
    phi0 = np.empty(nr)
    start = np.empty(nr, dtype=np.int64)
    for r in range(nr):
        i = r + 1
        if i < N:
            z[r] = 1.0 - i * i / (3.0 * N * N)
            nphi[r] = 4 * i
            phi0[r] = math.pi / (4.0 * i)
            start[r] = 2 * i * (i - 1)
        elif i <= 3 * N:
            z[r] = 4.0 / 3.0 - 2.0 * i / (3.0 * N)
            nphi[r] = 4 * N
            phi0[r] = (0.5 if (i - N) % 2 == 0 else 0.0) * math.pi / (2.0 * N)
            start[r] = 2 * N * (N - 1) + (i - N) * 4 * N
        else:
            ii = 4 * N - i
            z[r] = -(1.0 - ii * ii / (3.0 * N * N))
            nphi[r] = 4 * ii
            phi0[r] = math.pi / (4.0 * ii)
            start[r] = npix(N) - 2 * ii * (ii + 1)
    return z, nphi, phi0, start


def pixel_angles(nside):
    """(theta, phi) of every RING pixel."""
    z, nphi, phi0, start = ring_info(nside)
    th = np.empty(npix(nside))
    ph = np.empty(npix(nside))
    for r in range(len(z)):
        n = nphi[r]
        th[start[r]:start[r] + n] = math.acos(z[r])
        ph[start[r]:start[r] + n] = phi0[r] + 2.0 * math.pi * np.arange(n) / n
    return th, ph


# ----------------------------------------------------------------------------
# Legendre functions
# ----------------------------------------------------------------------------
def lambda_lm(L, x):
    """lambda[k, l, m] for x[k] (unscaled three-term recurrence in l)."""
    x = np.atleast_1d(np.asarray(x, dtype=np.float64))
    s = np.sqrt(np.maximum(0.0, 1.0 - x * x))
    lam = np.zeros((len(x), L + 1, L + 1))
    # lambda_mm = (-1)^m sqrt((2m+1)/(4pi) prod_{k<=m} (2k-1)/(2k)) sin^m
    pref = np.empty(L + 1)
    acc = 1.0 / FOURPI
    for m in range(L + 1):
        if m > 0:
            acc *= (2.0 * m - 1.0) / (2.0 * m)
        pref[m] = math.sqrt(acc * (2.0 * m + 1.0)) * (-1.0) ** m
    smin = s[s > 0].min() if np.any(s > 0) else 1.0
    assert L * math.log10(max(smin, 1e-300)) > -280, "oracle recurrence would underflow: use a smaller l_max"
    for m in range(L + 1):
        lmm = pref[m] * s ** m
        lam[:, m, m] = lmm
        if m + 1 <= L:
            lam[:, m + 1, m] = x * math.sqrt(2.0 * m + 3.0) * lmm
        for ell in range(m + 2, L + 1):
            a = math.sqrt((4.0 * ell * ell - 1.0) / (ell * ell - m * m))
            b = math.sqrt(((ell - 1.0) ** 2 - m * m) / (4.0 * (ell - 1.0) ** 2 - 1.0))
            lam[:, ell, m] = a * (x * lam[:, ell - 1, m] - b * lam[:, ell - 2, m])
    return lam


def spin2_F(L, x, lam=None):
    """(F1, F2)[k, l, m] of the spin-2 harmonics (+-2Y = (F1 +- F2) e^{im phi})."""
    x = np.atleast_1d(np.asarray(x, dtype=np.float64))
    if lam is None:
        lam = lambda_lm(L, x)
    ell = np.arange(L + 1, dtype=np.float64)[None, :, None]
    m = np.arange(L + 1, dtype=np.float64)[None, None, :]
    xx = x[:, None, None]
    is2 = 1.0 / (1.0 - xx * xx)
    c = np.zeros(L + 1)
    for l in range(2, L + 1):
        c[l] = 2.0 / math.sqrt((l - 1.0) * l * (l + 1.0) * (l + 2.0))
    c = c[None, :, None]
    with np.errstate(invalid="ignore", divide="ignore"):
        f = np.sqrt(np.maximum(0.0, (2 * ell + 1) / (2 * ell - 1) * (ell * ell - m * m)))
    f = np.where(ell >= 1, f, 0.0)
    lam1 = np.zeros_like(lam)
    lam1[:, 1:, :] = lam[:, :-1, :]
    F1 = c * (-((ell - m * m) * is2 + 0.5 * ell * (ell - 1)) * lam + f * xx * is2 * lam1)
    F2 = c * m * is2 * (-(ell - 1) * xx * lam + f * lam1)
    tri = (m <= ell)
    return np.where(tri, F1, 0.0), np.where(tri, F2, 0.0)


# ----------------------------------------------------------------------------
# transforms
# ----------------------------------------------------------------------------
def _cidx(L):
    ls, ms = [], []
    for m in range(L + 1):
        for l in range(m, L + 1):
            ls.append(l)
            ms.append(m)
    return np.array(ls), np.array(ms)


def _to_lm(alm, L):
    """healpy m-major complex vector -> dense [l, m] (zero above the diagonal)."""
    ls, ms = _cidx(L)
    A = np.zeros((L + 1, L + 1), dtype=np.complex128)
    A[ls, ms] = alm
    return A


def _from_lm(A, L):
    ls, ms = _cidx(L)
    return A[ls, ms].copy()


@functools.lru_cache(maxsize=2)
def _ring_exp(nside, L):
    """per ring the [nphi, L+1] table e^{i m phi_j} (cached per geometry: the
    oracle's transforms are direct sums, this only avoids recomputing them)."""
    z, nphi, phi0, start = ring_info(nside)
    m = np.arange(L + 1)
    out = []
    for r in range(len(z)):
        phi = phi0[r] + 2.0 * math.pi * np.arange(nphi[r]) / nphi[r]
        out.append(np.exp(1j * np.outer(phi, m)))
    return out


@functools.lru_cache(maxsize=2)
def _ring_legendre(nside, L):
    """(lambda, F1, F2)[ring, l, m] at the ring colatitudes (cached per geometry)."""
    z = ring_info(nside)[0]
    lam = lambda_lm(L, z)
    F1, F2 = spin2_F(L, z, lam)
    for a in (lam, F1, F2):
        a.flags.writeable = False
    return lam, F1, F2


def _ring_sum(F, nside):
    """map pixels from per-ring F[ring, m]: sum_m c_m Re[F_m e^{i m phi_j}]."""
    z, nphi, phi0, start = ring_info(nside)
    L = F.shape[1] - 1
    out = np.empty(npix(nside))
    cm = np.full(L + 1, 2.0)
    cm[0] = 1.0
    E = _ring_exp(nside, L)
    for r in range(len(z)):
        out[start[r]:start[r] + nphi[r]] = (E[r] @ (cm * F[r])).real
    return out


def _ring_phase(mp, nside, L):
    """Phi[ring, m] = sum_j map_j e^{-i m phi_j}."""
    z, nphi, phi0, start = ring_info(nside)
    P = np.empty((len(z), L + 1), dtype=np.complex128)
    E = _ring_exp(nside, L)
    for r in range(len(z)):
        P[r] = E[r].conj().T @ mp[start[r]:start[r] + nphi[r]]
    return P


def alm2map(alms, nside, lmax):
    """alms: complex [L lm] (spin 0, T only) or [3, nlm] (T, E, B -> T, Q, U)."""
    alms = np.asarray(alms)
    L = lmax
    lam, F1, F2 = _ring_legendre(nside, L)
    if alms.ndim == 1:
        A = _to_lm(alms, L)
        F = np.einsum("rlm,lm->rm", lam, A)
        return _ring_sum(F, nside)
    AT, AE, AB = (_to_lm(a, L) for a in alms)
    T = _ring_sum(np.einsum("rlm,lm->rm", lam, AT), nside)
    Q = _ring_sum(-(np.einsum("rlm,lm->rm", F1, AE) + 1j * np.einsum("rlm,lm->rm", F2, AB)), nside)
    U = _ring_sum(-(np.einsum("rlm,lm->rm", F1, AB) - 1j * np.einsum("rlm,lm->rm", F2, AE)), nside)
    return np.stack([T, Q, U])


def map2alm(maps, nside, lmax, iter=0):
    """healpy.map2alm(..., iter=iter, use_weights=False) restated."""
    maps = np.asarray(maps, dtype=np.float64)
    L = lmax
    w = FOURPI / npix(nside)
    lam, F1, F2 = _ring_legendre(nside, L)

    def adj(mp):
        if mp.ndim == 1:
            P = _ring_phase(mp, nside, L)
            return _from_lm(w * np.einsum("rlm,rm->lm", lam, P), L)
        PT, PQ, PU = (_ring_phase(x, nside, L) for x in mp)
        aT = w * np.einsum("rlm,rm->lm", lam, PT)
        aE = -w * (np.einsum("rlm,rm->lm", F1, PQ) + 1j * np.einsum("rlm,rm->lm", F2, PU))
        aB = -w * (np.einsum("rlm,rm->lm", F1, PU) - 1j * np.einsum("rlm,rm->lm", F2, PQ))
        return np.stack([_from_lm(aT, L), _from_lm(aE, L), _from_lm(aB, L)])

    a = adj(maps)
    for _ in range(iter):
        a = a + adj(maps - alm2map(a, nside, L))
    return a


def sph_harm_closed(ell, m, theta, phi):
    """A few closed-form Y_lm (Condon-Shortley) for the known-answer tests."""
    ct, st = np.cos(theta), np.sin(theta)
    e = np.exp(1j * m * phi)
    table = {
        (0, 0): lambda: np.full_like(theta, 0.5 / math.sqrt(math.pi)) + 0j,
        (1, 0): lambda: math.sqrt(3.0 / FOURPI) * ct + 0j,
        (1, 1): lambda: -math.sqrt(3.0 / (8.0 * math.pi)) * st * e,
        (2, 0): lambda: math.sqrt(5.0 / (16.0 * math.pi)) * (3 * ct * ct - 1) + 0j,
        (2, 1): lambda: -math.sqrt(15.0 / (8.0 * math.pi)) * st * ct * e,
        (2, 2): lambda: math.sqrt(15.0 / (32.0 * math.pi)) * st * st * e,
    }
    return table[(ell, m)]()


def spin2_closed(ell, m, s, theta, phi):
    """Closed-form sY_lm for l = 2 (s = +-2, m = 0, 2)."""
    ct, st = np.cos(theta), np.sin(theta)
    e = np.exp(1j * m * phi)
    if (ell, m) == (2, 0):
        return math.sqrt(15.0 / (32.0 * math.pi)) * st * st + 0j
    if (ell, m) == (2, 2):
        base = (1.0 - ct) ** 2 if s == 2 else (1.0 + ct) ** 2
        return math.sqrt(5.0 / math.pi) / 8.0 * base * e
    raise KeyError((ell, m))
