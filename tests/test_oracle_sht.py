"""CPU: pin the SHT oracle (oracle/sht.py) by analytic known answers.

healpy is absent offline and no reference test holds an SHT output, so the
oracle's HEALPix conventions are pinned here by closed-form Y_lm and
+-2Y_lm, scipy.special.sph_harm_y, exact adjointness, and band-limited
round trips.  Parity against healpy itself is
unpinned."""
import math

import numpy as np
import pytest
import scipy.special as sps

from oracle import sht as O


def _complex_index(L, l, m):
    return m * (2 * L + 1 - m) // 2 + l


def test_ring_geometry():
    for N in (1, 2, 4, 8, 16):
        z, nphi, phi0, start = O.ring_info(N)
        assert nphi.sum() == O.npix(N)
        assert np.all(np.diff(z) < 0)
        assert start[0] == 0 and np.all(start[1:] == np.cumsum(nphi)[:-1])
        # equal-area: each pixel covers 4pi/Npix; ring z edges reproduce it
        np.testing.assert_allclose(z, -z[::-1], atol=1e-15)
        th, ph = O.pixel_angles(N)
        assert np.all((ph >= 0) & (ph < 2 * np.pi))


@pytest.mark.parametrize("ell,m", [(0, 0), (1, 0), (1, 1), (2, 0), (2, 1), (2, 2)])
def test_single_mode_closed_form(ell, m):
    N, L = 8, 6
    a = np.zeros(O._cidx(L)[0].shape[0], dtype=np.complex128)
    a[_complex_index(L, ell, m)] = 0.7 - 0.3j
    mp = O.alm2map(a, N, L)
    th, ph = O.pixel_angles(N)
    Y = O.sph_harm_closed(ell, m, th, ph)
    want = ((0.7 - 0.3j) * Y).real if m == 0 else 2.0 * ((0.7 - 0.3j) * Y).real
    np.testing.assert_allclose(mp, want, atol=1e-13)


def test_lambda_vs_scipy():
    L = 40
    x = np.array([0.93, 0.41, -0.12, -0.77])
    lam = O.lambda_lm(L, x)
    th = np.arccos(x)
    for ell in (0, 3, 17, 40):
        for m in range(0, ell + 1, 5):
            Y = sps.sph_harm_y(ell, m, th, np.zeros_like(th))
            np.testing.assert_allclose(lam[:, ell, m], Y.real, rtol=1e-12, atol=1e-14)


def test_spin2_closed_form():
    """Q + iU = -sum (a_E + i a_B) 2Y (HEALPix) for a_E,20 and a_B,22 modes."""
    N, L = 8, 4
    th, ph = O.pixel_angles(N)
    nlm = O._cidx(L)[0].shape[0]
    # pure E, m = 0: Q = -2Y_20, U = 0
    a = np.zeros((3, nlm), dtype=np.complex128)
    a[1, _complex_index(L, 2, 0)] = 1.0
    T, Q, U = O.alm2map(a, N, L)
    np.testing.assert_allclose(Q, -O.spin2_closed(2, 0, 2, th, ph).real, atol=1e-13)
    np.testing.assert_allclose(U, 0.0, atol=1e-13)
    np.testing.assert_allclose(T, 0.0, atol=1e-13)
    # pure B, m = 2, a_B = 1: Q + iU = -i [2Y_22 + 2Y_2,-2], 2Y_2,-2 = (-2Y_22)^*
    a = np.zeros((3, nlm), dtype=np.complex128)
    a[2, _complex_index(L, 2, 2)] = 1.0
    T, Q, U = O.alm2map(a, N, L)
    pq = -1j * (O.spin2_closed(2, 2, 2, th, ph) + np.conj(O.spin2_closed(2, 2, -2, th, ph)))
    np.testing.assert_allclose(Q, pq.real, atol=1e-13)
    np.testing.assert_allclose(U, pq.imag, atol=1e-13)


def _rand_alm(L, ncomp, rng):
    ls, ms = O._cidx(L)
    a = rng.standard_normal((ncomp, len(ls))) + 1j * rng.standard_normal((ncomp, len(ls)))
    a[:, ms == 0] = a[:, ms == 0].real
    return a


def _alm_dot(a, b, L):
    ls, ms = O._cidx(L)
    w = np.where(ms == 0, 1.0, 2.0)
    return float(np.sum(w * (a * np.conj(b)).real))


@pytest.mark.parametrize("pol", [False, True])
def test_adjointness(pol):
    """<alm2map(a), m> = <a, map2alm(m)> / w exactly (iter = 0)."""
    N, L = 8, 20
    rng = np.random.default_rng(5)
    nc = 3 if pol else 1
    a = _rand_alm(L, nc, rng)
    mp = rng.standard_normal((nc, O.npix(N)))
    if not pol:
        a, mp = a[0], mp[0]
    Am = O.alm2map(a, N, L)
    Atm = O.map2alm(mp, N, L) / (4 * np.pi / O.npix(N))
    lhs = float(np.sum(Am * mp))
    rhs = _alm_dot(np.atleast_2d(a), np.atleast_2d(Atm), L)
    assert abs(lhs - rhs) <= 1e-11 * (abs(lhs) + 1.0)


@pytest.mark.parametrize("pol", [False, True])
def test_band_limited_round_trip(pol):
    """map2alm(alm2map(a), iter=3) ~ a for l <= 1.5 N_side; error shrinks with iter."""
    N = 8
    L = 12
    rng = np.random.default_rng(7)
    a = _rand_alm(L, 3 if pol else 1, rng)
    if pol:
        a[:, O._cidx(L)[0] < 2] = 0.0
    else:
        a = a[0]
    mp = O.alm2map(a, N, L)
    e0 = np.abs(O.map2alm(mp, N, L, iter=0) - a).max()
    e3 = np.abs(O.map2alm(mp, N, L, iter=3) - a).max()
    assert e3 < 1e-4 * np.abs(a).max()
    assert e3 < e0


# ---- the C++/OpenMP SHT of the CPU baseline (oracle/sht_cpu.cpp) ------------------------
@pytest.mark.parametrize("N,L", [(8, 16), (16, 47), (32, 64)])
def test_sht_cpu_matches_dense_oracle(N, L):
    """oracle/sht_cpu.cpp (ring FFTs, scaled recurrence, ring-pair blocks) equals the
    dense direct sums of oracle/sht.py: spin 0, spin 2 alone (comps 2) and TEB,
    alm2map and map2alm with iter 0 and 3."""
    from oracle import sht_cpu as C
    rng = np.random.default_rng(N + L)
    ls, ms = O._cidx(L)
    a = rng.normal(size=(3, len(ls))) + 1j * rng.normal(size=(3, len(ls)))
    a[:, ms == 0] = a[:, ms == 0].real
    a[1:, ls < 2] = 0
    want = O.alm2map(a, N, L)
    tol = 1e-12 * np.abs(want).max()
    np.testing.assert_allclose(C.alm2map(a, N, L), want, rtol=0, atol=tol)
    np.testing.assert_allclose(C.alm2map(a[0], N, L), want[0], rtol=0, atol=tol)
    np.testing.assert_allclose(C.alm2map(a[1:], N, L), want[1:], rtol=0, atol=tol)
    mp = rng.normal(size=(3, 12 * N * N))
    for it in (0, 3):
        want = O.map2alm(mp, N, L, iter=it)
        tol = 1e-12 * np.abs(want).max()
        np.testing.assert_allclose(C.map2alm(mp, N, L, iter=it), want, rtol=0, atol=tol)
        np.testing.assert_allclose(C.map2alm(mp[1:], N, L, iter=it), want[1:], rtol=0, atol=tol)
        np.testing.assert_allclose(C.map2alm(mp[0], N, L, iter=it), want[0], rtol=0, atol=tol)
