"""Properties of the oracle restatement (and therefore of the spec the HIP path
is tested against): RNG known-answer tests, TEB -> EB reduction, inverse-Wishart
p=1 -> inverse-Gamma reduction, truncated-normal inverse CDF vs scipy, the
per-l decomposition of the all_sph likelihood vs the full-sky sum."""
import math

import numpy as np
import pytest
from scipy import stats

from oracle import harmonic as H
from oracle.cpu_baseline import _loglik_full
from tests._util import make_problem


def _hex(w):
    return " ".join("%08x" % int(x) for x in w)


def test_philox_known_answers():
    """Random123 kat_vectors for philox4x32-10."""
    f = H.philox4x32_10
    assert _hex(f(0, 0, 0, 0, 0, 0)) == "6627e8d5 e169c58d bc57ac4c 9b00dbd8"
    m = 0xFFFFFFFF
    assert _hex(f(m, m, m, m, m, m)) == "408f276d 41c83b0e a20bc7c6 6d5451fd"
    assert _hex(f(0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344, 0xa4093822, 0x299f31d0)) == \
        "d16cfe09 94fdcceb 5001e420 24126ea1"


def test_native_normals_are_standard():
    z = np.concatenate([H.cr_normals(11, c, 3, 0, f, 160) for c in range(2) for f in range(3)])
    n = len(z)
    assert abs(z.mean()) < 5 / math.sqrt(n)
    assert abs(z.var() - 1) < 6 * math.sqrt(2 / n)
    assert stats.kstest(z, "norm").pvalue > 1e-4


def test_gamma_native_moments():
    k0, k1 = H.chain_key(5, 0)
    for alpha in (0.5, 1.0, 7.5, 300.0):
        g = np.array([H.gamma_native(alpha, k0, k1, b, 0, 1) for b in range(3000)])
        assert abs(g.mean() - alpha) < 6 * math.sqrt(alpha / len(g))
        assert stats.kstest(g, "gamma", args=(alpha,)).pvalue > 1e-4


def test_teb_reduces_to_eb():
    """With TT = TE = 0 the TEB operators of E and B equal the EB ones."""
    L = 30
    m3, init3 = make_problem(L, 16, 3, seed=1)
    m2, _ = make_problem(L, 16, 2, seed=1)
    un3 = m3.unfold(init3)
    un3[0] = 0.0
    un3[3] = 0.0
    un2 = un3[[1, 2]]
    m2.bl = m3.bl
    m2.noise_var = [m3.noise_var[1], m3.noise_var[2]]
    m2.kappa = [m3.kappa[1], m3.kappa[2]]
    for fn in (H.centered_params, H.noncentered_params):
        M3, L3 = fn(m3, un3)
        M2, L2 = fn(m2, un2)
        np.testing.assert_allclose(M3[:, 1, 1], M2[:, 0, 0], rtol=1e-13, atol=1e-300)
        np.testing.assert_allclose(M3[:, 2, 2], M2[:, 1, 1], rtol=1e-13, atol=1e-300)
        np.testing.assert_allclose(L3[:, 1, 1], L2[:, 0, 0], rtol=1e-13, atol=1e-300)
        np.testing.assert_allclose(L3[:, 2, 2], L2[:, 1, 1], rtol=1e-13, atol=1e-300)
        np.testing.assert_allclose(M3[:, 1, 0], 0.0, atol=1e-300)


def test_centered_cr_is_the_gaussian_posterior():
    """s = M d + L z has mean Sigma B N^-1 d and covariance Sigma = (C^+ + P)^-1."""
    L = 12
    m, init = make_problem(L, 8, 3, seed=2)
    un = m.unfold(init)
    M, Lc = H.centered_params(m, un)
    C = H.cov_blocks(m, un)
    for ell in (2, 7, 12):
        Q = np.linalg.inv(C[ell]) + np.diag([m.bl[ell] ** 2 * k for k in m.kappa])
        S = np.linalg.inv(Q)
        np.testing.assert_allclose(Lc[ell] @ Lc[ell].T, S, rtol=1e-10, atol=1e-18)
        np.testing.assert_allclose(M[ell], S @ np.diag([m.bl[ell] * k for k in m.kappa]), rtol=1e-10, atol=1e-18)


def test_inverse_wishart_p1_is_inverse_gamma():
    """IW(nu, Psi) for p = 1 is IG(nu/2, Psi/2): the alpha/beta of CenteredGibbs.py:62-76."""
    L = 20
    m, _ = make_problem(L, 16, 2, seed=3)
    ss = np.random.RandomState(0).uniform(1, 2, size=(2, 2, L + 1))
    chat = H.centered_betas(m, ss)
    alpha, beta = H.invgamma_params(m, "EE", chat["EE"])
    ell = np.arange(L + 1.0)
    b = m.bins["EE"]
    for i in range(2, len(b) - 1):
        sl = slice(b[i], b[i + 1])
        nu = np.sum(2 * ell[sl] + 1) - 2
        psi = np.sum(ell[sl] * (ell[sl] + 1) / (2 * np.pi) * ss[0, 0, sl])
        assert alpha[i] == pytest.approx(nu / 2)
        assert beta[i] == pytest.approx(psi / 2)


def test_truncnorm_ppf_matches_scipy():
    rng = np.random.RandomState(4)
    q = rng.uniform(size=2000)
    a = -rng.exponential(5.0, size=2000)
    np.testing.assert_allclose(H.truncnorm_ppf_std(q, a), stats.truncnorm.ppf(q, a, np.inf), rtol=1e-9, atol=1e-12)


def test_block_likelihood_decomposition_matches_full_sum():
    """sum_l f_l (per-l sufficient statistics) == full-sky likelihood up to the
    constant sum d^2 -- the identity that makes every MH block O(width)."""
    L = 20
    for F in (2, 3):
        m, init = make_problem(L, 16, F, seed=5)
        un = m.unfold(init)
        rng = np.random.RandomState(6)
        s = rng.normal(size=(F, (L + 1) ** 2))
        st = H.sweep_stats(m, s, m.d_alm)
        full = _loglik_full(m, un, s, H.slot_ell(L))
        const = -0.5 * sum(m.kappa[f] * np.sum(m.d_alm[f] ** 2) for f in range(F))
        np.testing.assert_allclose(np.sum(H.nc_loglik_terms(m, un, st)) + const, full, rtol=1e-11)


def test_mh_blocks_of_one_spectrum_are_independent():
    """Accepting one block never changes another block's acceptance ratio."""
    L = 24
    m, init = make_problem(L, 16, 2, seed=7)
    un = m.unfold(init)
    st = H.sweep_stats(m, np.random.RandomState(1).normal(size=(2, (L + 1) ** 2)), m.d_alm)
    f0 = H.nc_loglik_terms(m, un, st)
    new = {k: v.copy() for k, v in init.items()}
    new["BB"][5] *= 1.3
    f1 = H.nc_loglik_terms(m, m.unfold(new), st)
    changed = np.nonzero(f1 != f0)[0]
    b = m.bins["BB"]
    assert set(changed) <= set(range(b[5], b[6]))


def test_cpu_baseline_ports_agree():
    """The two CPU baselines of bench.py (oracle/cpu_baseline.py) are the same
    chain: the reference-structured port (full-sky likelihood per block) and the
    algorithm-matched port (per-l statistics) take the same decisions from the
    same numpy draws (EB and TEB)."""
    from oracle import cpu_baseline as CB
    from tests._util import make_problem
    for F in (2, 3):
        m, init = make_problem(24, 16, F, seed=4)
        np.random.seed(5)
        a = CB.nc_iteration(m, init)
        np.random.seed(5)
        b = CB.nc_iteration_matched(m, init)
        for s in m.spectra:
            np.testing.assert_allclose(a[s], b[s], rtol=1e-12)
