"""numpy restatement of the MASKED constrained-realization samplers (TEST INFRASTRUCTURE).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import
this module; the product path never does.

Restates (Gabriel-Ducrocq/GibbsSampler, EB / "polarization" class):
  * the constructor's constants         CenteredGibbs.py:258-306
      N^-1 = mask / noise_pol, mu = max(N^-1) + 1e-14, second_part_grad =
      b * complex_to_real(map2alm([0, Q N^-1, U N^-1], iter=0)) * Npix/4pi
  * sample_gibbs_change_variable (a9)   CenteredGibbs.py:676-729
  * overrelaxation_sampler (a10)        CenteredGibbs.py:733-825
  * compute_gradient_mala / propose_new_mala / compute_log_proposal /
    compute_log_density / sample_mala (a11)   CenteredGibbs.py:494-603
  * the dispatch ladder of sample (a12)  CenteredGibbs.py:828-850
with the build's SHT oracle (oracle/sht.py) in place of healpy.  Pinned by
tests/golden/reference_masked_eb_*.npz, produced by running the reference
itself (tools/gen_golden_masked.py) with that same SHT behind its healpy
import: these fixtures pin the samplers' algebra, scalings and draw order,
not healpy's transform (parity unpinned).

TEB generalisation (not in the reference): T uses its own N_T^-1 and
mu_T = max(N_T^-1) + 1e-14; the s|v draw is the per-l 3x3 centered block of
oracle.harmonic with kappa_f = mu_f / w; over-relaxation uses the Cholesky
factor of that block.

Draws come from a ``Draws`` source: ``ReplayDraws`` consumes numpy's legacy
global stream in the reference's order (parity with the fixtures);
``NativeDraws`` restates the device's counter-based Philox streams.
"""
import math

import numpy as np

from . import harmonic as H
from . import sht as O

FOURPI = 4.0 * math.pi
TAG_AUX_V = 8        # pixel normals of v | s; c0 = pixel, c1 = map (0 T, 1 Q, 2 U)
TAG_MALA_U = 9       # MALA accept uniform
TAG_RJ_U = 10        # RJPO accept uniform (c0 = c1 = 0)
SUB_S = 16           # CR substep base of the s | v draws: SUB_S + 2k (+1: second OR draw)
SUB_V_INIT = 255     # substep of the over-relaxation's initial v | s
SUB_MALA = 200       # CR substep of the MALA proposal normals (+ call index)


class ReplayDraws:
    """numpy legacy global RNG, in the reference's order."""

    def __init__(self, seed=None):
        if seed is not None:
            np.random.seed(seed)

    def pixel_normals(self, nmaps, npix, **kw):
        return np.stack([np.random.normal(size=npix) for _ in range(nmaps)])

    def slot_normals(self, nfields, nreal, **kw):
        return np.stack([np.random.normal(size=nreal) for _ in range(nfields)])

    def uniform(self, **kw):
        return np.random.uniform()


class NativeDraws:
    """The device's Philox4x32-10 streams (gibbssampler_amd/csrc/gs_masked.hip)."""

    def __init__(self, seed, chain, iteration, L, npix):
        self.seed, self.chain, self.it, self.L, self.npix = int(seed), int(chain), int(iteration), L, npix

    def pixel_normals(self, nmaps, npix, maps=(1, 2), substep=0):
        k0, k1 = H.chain_key(self.seed, self.chain)
        p = np.arange(npix, dtype=np.uint64)
        out = []
        for f in maps:
            w = H.philox4x32_10(p, f, TAG_AUX_V | (substep << 8), self.it, k0, k1)
            out.append(H.box_muller(*w)[0])
        return np.stack(out)

    def slot_normals(self, nfields, nreal, substep=0):
        return np.stack([H.cr_normals(self.seed, self.chain, self.it, substep, f, self.L) for f in range(nfields)])

    def uniform(self, substep=0, tag=TAG_MALA_U):
        k0, k1 = H.chain_key(self.seed, self.chain)
        return H._uniform1(k0, k1, 0, substep, tag, self.it)


class MaskedModel:
    """Pixel-domain data and noise of one masked problem.

    maps: [3, Npix] (T, Q, U); inv_noise: [3, Npix] mask-multiplied N^-1
    (T row ignored for nfields = 2)."""

    def __init__(self, L, nside, nfields, bl, maps, inv_noise, mu_eps=1e-14, adj_iter=0, sht=None):
        self.L, self.nside, self.F = int(L), int(nside), int(nfields)
        # the transform module (alm2map / map2alm with oracle.sht's interface): the
        # dense oracle by default; oracle.sht_cpu for the CPU baseline at full size
        self.sht = O if sht is None else sht
        self.adj_iter = int(adj_iter)
        self.Npix = 12 * self.nside ** 2
        self.w = FOURPI / self.Npix
        self.bl = np.asarray(bl, dtype=np.float64)
        self.maps = np.asarray(maps, dtype=np.float64)
        self.inv_noise = np.asarray(inv_noise, dtype=np.float64)
        # CenteredGibbs.py:276 (pol, 1e-14); TEB: the same rule for T; TT (nfields 1):
        # ConstrainedRealization.py:44 (1e-7)
        self.mu = np.array([self.inv_noise[k].max() + mu_eps for k in range(3)])
        self.slot_ell = H.slot_ell(self.L)

    # fields -> map rows: F=1: T; F=2: E,B <-> Q,U (rows 1,2); F=3: T,E,B <-> T,Q,U
    @property
    def rows(self):
        return {1: (0,), 2: (1, 2), 3: (0, 1, 2)}[self.F]

    def synth(self, s_real):
        """maps of b * s (s real layout [F, NR]) -> [F, Npix] for the field rows."""
        ls = O._cidx(self.L)[0]
        if self.F == 1:          # temperature only: the spin-0 transform alone
            return self.sht.alm2map(H.real_to_complex(s_real[0], self.L) * self.bl[ls], self.nside, self.L)[None]
        a = np.zeros((3, ls.shape[0]), dtype=np.complex128)
        for k, r in enumerate(self.rows):
            a[r] = H.real_to_complex(s_real[k], self.L) * self.bl[ls]
        m = self.sht.alm2map(a, self.nside, self.L)
        return np.stack([m[r] for r in self.rows])

    def analysis(self, mp, iter=0):
        """complex_to_real(map2alm(maps, iter)) for the field rows: [F, NR]."""
        if self.F == 1:          # temperature only: the spin-0 transform alone
            return H.complex_to_real(self.sht.map2alm(np.asarray(mp)[0], self.nside, self.L, iter=iter), self.L)[None]
        full = np.zeros((3, self.Npix))
        for k, r in enumerate(self.rows):
            full[r] = mp[k]
        a = self.sht.map2alm(full, self.nside, self.L, iter=iter)
        return np.stack([H.complex_to_real(a[r], self.L) for r in self.rows])

    def second_part_grad(self):
        """b A^T N^-1 d (CenteredGibbs.py:298-306; TT: adjoint_synthesis_hp, iter 3)."""
        nd = np.stack([self.inv_noise[r] * self.maps[r] for r in self.rows])
        return self.analysis(nd, self.adj_iter) * (self.Npix / FOURPI) * self.bl[self.slot_ell][None]

    def aux_model(self, bins):
        """oracle.harmonic Model whose kappa_f = mu_f / w (the s | v block)."""
        mu = [self.mu[r] for r in self.rows]
        return H.Model(self.L, self.nside, self.F, self.bl, [1.0 / m for m in mu], bins)


# ----------------------------------------------------------------------------
# a9 / a10: auxiliary-variable CR
# ----------------------------------------------------------------------------
def _v_given_s(mm, s, z, v_old=None, alpha=None):
    """v | s  (CenteredGibbs.py:693-700): v = gamma A b s + sqrt(gamma) z,
    gamma = mu - N^-1; over-relaxed (801-802): v' = m + alpha (v - m) +
    sqrt(1 - alpha^2) sqrt(gamma) z."""
    mp = mm.synth(s)
    out = []
    for k, r in enumerate(mm.rows):
        gam = mm.mu[r] - mm.inv_noise[r]
        mean = gam * mp[k]
        if alpha is None:
            out.append(z[k] * np.sqrt(gam) + mean)
        else:
            out.append(mean + alpha * (v_old[k] - mean) + math.sqrt(1 - alpha ** 2) * z[k] * np.sqrt(gam))
    return np.stack(out)


def _s_given_v(mm, dl_unbinned, v, z, s_old=None, alpha=None):
    """s | v  (CenteredGibbs.py:703-726): per slot (EB) or per-l block (TEB)
    var_s = (C^+ + (mu/w) b^2)^-1, mean = var_s b map2alm(v + N^-1 d)/w."""
    rhs = np.stack([v[k] + mm.inv_noise[r] * mm.maps[r] for k, r in enumerate(mm.rows)])
    r_real = mm.analysis(rhs, mm.adj_iter)
    ell = mm.slot_ell
    if mm.F != 3:
        out = []
        var = H.var_from_dl(dl_unbinned)
        for k, r in enumerate(mm.rows):
            var_s = 1.0 / ((mm.mu[r] / mm.w) * mm.bl[ell] ** 2 + H.inv_var(var[k][ell]))
            mean = var_s * (r_real[k] / mm.w * mm.bl[ell])
            if alpha is None:
                out.append(z[k] * np.sqrt(var_s) + mean)
            else:
                out.append(mean + alpha * (s_old[k] - mean) + math.sqrt(1 - alpha ** 2) * z[k] * np.sqrt(var_s))
        return np.stack(out)
    model = mm.aux_model({s: np.arange(mm.L + 2) for s in H.SPECTRA[3]})
    M, Lc = H.centered_params(model, dl_unbinned)
    d_eff = np.stack([r_real[k] / mm.mu[r] for k, r in enumerate(mm.rows)])
    mean = H.cr_apply(model, M, np.zeros_like(M), d_eff, np.zeros_like(d_eff))
    fl = H.cr_apply(model, np.zeros_like(M), Lc, d_eff, z)
    if alpha is None:
        return mean + fl
    return mean + alpha * (s_old - mean) + math.sqrt(1 - alpha ** 2) * fl


def aux_variable(mm, dl_unbinned, s_old, n_gibbs, draws):
    """sample_gibbs_change_variable (a9): n_gibbs x (v | s, s | v); accept 1."""
    s = np.array(s_old, dtype=np.float64)
    nr = (mm.L + 1) ** 2
    for k in range(n_gibbs):
        zv = draws.pixel_normals(mm.F, mm.Npix, maps=mm.rows, substep=k)
        v = _v_given_s(mm, s, zv)
        zs = draws.slot_normals(mm.F, nr, substep=SUB_S + 2 * k)
        s = _s_given_v(mm, dl_unbinned, v, zs)
    return s, 1


def overrelaxation(mm, dl_unbinned, s_old, n_gibbs, draws, alpha=-0.995):
    """overrelaxation_sampler (a10): v | s plain, then n_gibbs x
    (s | v, v | s, s | v) all over-relaxed; accept 1."""
    s = np.array(s_old, dtype=np.float64)
    nr = (mm.L + 1) ** 2
    v = _v_given_s(mm, s, draws.pixel_normals(mm.F, mm.Npix, maps=mm.rows, substep=SUB_V_INIT))
    for k in range(n_gibbs):
        s = _s_given_v(mm, dl_unbinned, v, draws.slot_normals(mm.F, nr, substep=SUB_S + 2 * k), s_old=s, alpha=alpha)
        v = _v_given_s(mm, s, draws.pixel_normals(mm.F, mm.Npix, maps=mm.rows, substep=k), v_old=v, alpha=alpha)
        s = _s_given_v(mm, dl_unbinned, v, draws.slot_normals(mm.F, nr, substep=SUB_S + 2 * k + 1), s_old=s,
                       alpha=alpha)
    return s, 1


# ----------------------------------------------------------------------------
# a11: MALA (EB, CenteredGibbs.py:494-603)
# ----------------------------------------------------------------------------
def mala_sigma(mm, dl_unbinned, noise_pol0):
    """sigma = 1/((Npix/(noise_pol[0] 4pi)) b^2 + C^-1) per slot (571-572)."""
    var = H.var_from_dl(dl_unbinned)
    ell = mm.slot_ell
    return np.stack([1.0 / ((mm.Npix / (noise_pol0 * FOURPI)) * mm.bl[ell] ** 2 + H.inv_var(var[k][ell]))
                     for k in range(mm.F)])


def mala_gradient(mm, dl_unbinned, s, g2):
    """grad = -C^-1 s - b A^T N^-1 A b s + b A^T N^-1 d; also returns A b s."""
    var = H.var_from_dl(dl_unbinned)
    ell = mm.slot_ell
    pix = mm.synth(s)
    nq = np.stack([mm.inv_noise[r] * pix[k] for k, r in enumerate(mm.rows)])
    second = -(mm.analysis(nq) / mm.w) * mm.bl[ell][None]
    first = -np.stack([H.inv_var(var[k][ell]) * s[k] for k in range(mm.F)])
    return first + second + g2, pix


def mala_log_density(mm, dl_unbinned, s, pix, g2):
    var = H.var_from_dl(dl_unbinned)
    ell = mm.slot_ell
    t1 = sum(-0.5 * np.sum(H.inv_var(var[k][ell]) * s[k] ** 2) for k in range(mm.F))
    t2 = sum(-0.5 * np.sum(pix[k] ** 2 * mm.inv_noise[r]) for k, r in enumerate(mm.rows))
    return t1 + t2 + float(np.sum(s * g2))


def mala_log_proposal(s_new, s_old, grad_old, sigma, tau):
    return float(np.sum(-0.5 * (s_new - s_old - tau * sigma * grad_old) ** 2 / (2 * tau * sigma)))


def mala(mm, dl_unbinned, s_old, draws, noise_pol0, tau=0.02, call=0):
    """sample_mala: one proposal, accept/reject; returns (s, accept, log_ratio)."""
    s_old = np.array(s_old, dtype=np.float64)
    g2 = mm.second_part_grad()
    sigma = mala_sigma(mm, dl_unbinned, noise_pol0)
    grad_old, pix_old = mala_gradient(mm, dl_unbinned, s_old, g2)
    z = draws.slot_normals(mm.F, (mm.L + 1) ** 2, substep=SUB_MALA + call)
    s_new = s_old + tau * sigma * grad_old + np.sqrt(2 * tau * sigma) * z
    grad_new, pix_new = mala_gradient(mm, dl_unbinned, s_new, g2)
    lr = (mala_log_density(mm, dl_unbinned, s_new, pix_new, g2) + mala_log_proposal(s_old, s_new, grad_new, sigma, tau)
          - (mala_log_density(mm, dl_unbinned, s_old, pix_old, g2)
             + mala_log_proposal(s_new, s_old, grad_old, sigma, tau)))
    u = draws.uniform(substep=call)
    if math.log(u) < lr:
        return s_new, 1, lr
    return s_old, 0, lr


def sample_dispatch(mm, dl_unbinned, s_old, draws, gibbs_cr, overrelaxation_flag, ula, n_gibbs, noise_pol0,
                    alpha=-0.995, tau=0.02):
    """CenteredGibbs.py:828-850 for a masked run with a previous map."""
    if gibbs_cr and overrelaxation_flag:
        return overrelaxation(mm, dl_unbinned, s_old, n_gibbs, draws, alpha)
    if gibbs_cr and not ula:
        return aux_variable(mm, dl_unbinned, s_old, n_gibbs, draws)
    if gibbs_cr and ula:
        s_mid, _ = aux_variable(mm, dl_unbinned, s_old, n_gibbs, draws)
        s, acc, _ = mala(mm, dl_unbinned, s_mid, draws, noise_pol0, tau)
        return s, acc
    if ula:
        s, acc, _ = mala(mm, dl_unbinned, s_old, draws, noise_pol0, tau)
        return s, acc
    raise NotImplementedError("PCG CR (sample_mask, qcinv) is SURVEY.md 8 row f1")


# ----------------------------------------------------------------------------
# f1: PCG constrained realisation (CenteredGibbs.py:448-491)
# ----------------------------------------------------------------------------
SUB_PCG_S = 250       # CR substep of the PCG's C^-1/2 slot normals
SUB_PCG_V = 254       # TAG_AUX_V substep of the PCG's pixel normals


def _prior_pinv_apply(mm, dl_unbinned, x, half=False):
    """C^+ x per slot (EB: inv_var; TEB: 2x2 TE pseudo-inverse + BB); with
    half=True the factor (A^+)^T (covariance C^+) used for the C^-1/2 draw."""
    ell = mm.slot_ell
    if mm.F != 3:
        var = H.var_from_dl(dl_unbinned)
        f = (lambda v: np.sqrt(H.inv_var(v))) if half else H.inv_var
        return np.stack([f(var[k][ell]) * x[k] for k in range(mm.F)])
    model = H.Model(mm.L, mm.nside, 3, mm.bl, [1.0, 1.0, 1.0], {s: np.arange(mm.L + 2) for s in H.SPECTRA[3]})
    A = H.cov_chol(model, dl_unbinned)
    Ai = H.chol_pinv(A)                                    # A^+ (lower)
    out = np.zeros_like(x)
    if half:                                               # (A^+)^T x
        Ms = np.transpose(Ai, (0, 2, 1))
        for f in range(3):
            for g in range(3):
                out[f] += Ms[ell, f, g] * x[g]
        return out
    P = np.einsum("lji,ljk->lik", Ai, Ai)                  # C^+ = (A^+)^T A^+
    for f in range(3):
        for g in range(3):
            out[f] += P[ell, f, g] * x[g]
    return out


def pcg_fluctuation(mm, dl_unbinned, z_pix, z_slot):
    """b_fluctuations (CenteredGibbs.py:467-482): b * adjoint_synthesis_hp(sqrt(N^-1) z_pix)
    (utils.py:79-111: map2alm iter=3 times Npix/4pi) + C^-1/2 z_slot."""
    y = np.stack([np.sqrt(mm.inv_noise[r]) * z_pix[k] for k, r in enumerate(mm.rows)])
    full = np.zeros((3, mm.Npix))
    for k, r in enumerate(mm.rows):
        full[r] = y[k]
    a = mm.sht.map2alm(full, mm.nside, mm.L, iter=3)
    adj = np.stack([H.complex_to_real(a[r], mm.L) for r in mm.rows]) * (mm.Npix / FOURPI)
    return adj * mm.bl[mm.slot_ell][None] + _prior_pinv_apply(mm, dl_unbinned, z_slot, half=True)


def pcg_operator(mm, dl_unbinned, x):
    """Q x = C^+ x + b A^T N^-1 A b x, A^T = map2alm(iter=0) / w (exact adjoint)."""
    pix = mm.synth(x)
    nq = np.stack([mm.inv_noise[r] * pix[k] for k, r in enumerate(mm.rows)])
    return _prior_pinv_apply(mm, dl_unbinned, x) + (mm.analysis(nq) / mm.w) * mm.bl[mm.slot_ell][None]


def pcg_solve(mm, dl_unbinned, rhs, tol=1e-12, maxiter=2000, x0=None):
    """Preconditioned CG on Q x = rhs; preconditioner (C^+ + diag(b^2 nbar/w))^-1
    per l (nbar = mean N^-1 of the field's map).  Stops at |r| <= tol |rhs|."""
    nbar = [mm.inv_noise[r].mean() for r in mm.rows]
    model = H.Model(mm.L, mm.nside, mm.F, mm.bl, [1.0 / n if n > 0 else 1e300 for n in nbar],
                    {s: np.arange(mm.L + 2) for s in H.SPECTRA[mm.F]})
    _, Lc = H.centered_params(model, dl_unbinned)
    ell = mm.slot_ell

    def prec(r):
        t = np.zeros_like(r)
        for f in range(mm.F):                      # L^T r
            for g in range(mm.F):
                t[f] += Lc[ell, g, f] * r[g]
        out = np.zeros_like(r)
        for f in range(mm.F):                      # L (L^T r)
            for g in range(mm.F):
                out[f] += Lc[ell, f, g] * t[g]
        return out

    x = np.zeros_like(rhs) if x0 is None else np.array(x0, dtype=np.float64)
    r = rhs - pcg_operator(mm, dl_unbinned, x)
    z = prec(r)
    p = z.copy()
    rz = float(np.sum(r * z))
    bn = float(np.sqrt(np.sum(rhs * rhs)))
    it = 0
    while it < maxiter and np.sqrt(np.sum(r * r)) > tol * bn:
        q = pcg_operator(mm, dl_unbinned, p)
        alpha = rz / float(np.sum(p * q))
        x = x + alpha * p
        r = r - alpha * q
        z = prec(r)
        rz_new = float(np.sum(r * z))
        p = z + (rz_new / rz) * p
        rz = rz_new
        it += 1
    return x, it


def pcg_sample(mm, dl_unbinned, draws, tol=1e-12, maxiter=2000):
    """sample_mask: rhs = b A^T N^-1 d + fluctuations; x = Q^-1 rhs; accept 1."""
    z_pix = draws.pixel_normals(mm.F, mm.Npix, maps=mm.rows, substep=SUB_PCG_V)
    z_slot = draws.slot_normals(mm.F, (mm.L + 1) ** 2, substep=SUB_PCG_S)
    rhs = mm.second_part_grad() + pcg_fluctuation(mm, dl_unbinned, z_pix, z_slot)
    x, it = pcg_solve(mm, dl_unbinned, rhs, tol, maxiter)
    return x, 1, it


def rj_sample(mm, dl_unbinned, draws, s_old, tol=1e-12, maxiter=2000):
    """sample_mask_rj (CenteredGibbs.py:606-674): the rhs of sample_mask (same
    draws, :622-643), the PCG started from -s_old (:645-650), then
    log_proba = -sum (rhs - Q x) . (s_old - x) (:652-669) and accept when
    log u < log_proba (:670; the uniform drawn after the normals).
    Returns (map, accept, log_proba, CG iterations)."""
    z_pix = draws.pixel_normals(mm.F, mm.Npix, maps=mm.rows, substep=SUB_PCG_V)
    z_slot = draws.slot_normals(mm.F, (mm.L + 1) ** 2, substep=SUB_PCG_S)
    rhs = mm.second_part_grad() + pcg_fluctuation(mm, dl_unbinned, z_pix, z_slot)
    u = draws.uniform(tag=TAG_RJ_U)
    x, it = pcg_solve(mm, dl_unbinned, rhs, tol, maxiter, x0=-np.asarray(s_old, dtype=np.float64))
    r = rhs - pcg_operator(mm, dl_unbinned, x)
    lp = -float(np.sum(r * (s_old - x)))
    if math.log(u) < lp:
        return x, 1, lp, it
    return np.array(s_old, dtype=np.float64), 0, lp, it


# ----------------------------------------------------------------------------
# f2: pixel-domain non-centered likelihood (NonCenteredGibbs.py:333-355)
# ----------------------------------------------------------------------------
def nc_map(mm, dl_unbinned, s_nc):
    """A b C^1/2(D) s_nc for the field rows (EB: sqrt(var) per slot; TEB: chol(C))."""
    if mm.F != 3:
        var = H.var_from_dl(dl_unbinned)
        s = np.stack([np.sqrt(var[k][mm.slot_ell]) * s_nc[k] for k in range(mm.F)])
    else:
        model = H.Model(mm.L, mm.nside, 3, mm.bl, [1.0] * 3, {x: np.arange(mm.L + 2) for x in H.SPECTRA[3]})
        A = H.cov_chol(model, dl_unbinned)
        s = np.zeros_like(s_nc)
        for f in range(3):
            for g in range(3):
                s[f] += A[mm.slot_ell, f, g] * s_nc[g]
    return mm.synth(s)


def nc_loglik_pixel(mm, dl_unbinned, s_nc):
    """-1/2 sum_pix N^-1 [(Q_d - Q)^2 + (U_d - U)^2]  (TEB adds the T row)."""
    mp = nc_map(mm, dl_unbinned, s_nc)
    return -0.5 * sum(float(np.sum((mm.maps[r] - mp[k]) ** 2 * mm.inv_noise[r])) for k, r in enumerate(mm.rows))


def pixel_mh(mm, model, dl_binned_old, s_nc, seed=0, chain=0, iteration=0, u_prop=None, u_accept=None, n_iter=1):
    """PolarizationNonCenteredClsSampler.sample with all_sph=False (401-445):
    the truncated-normal proposals and block loop of oracle.harmonic.nc_mh,
    each block scored by the full pixel-domain likelihood."""
    return H.nc_mh(model, dl_binned_old, None, seed=seed, chain=chain, iteration=iteration, u_prop=u_prop,
                   u_accept=u_accept, n_iter=n_iter, loglik=lambda dl: nc_loglik_pixel(mm, dl, s_nc))


def noncentre(mm, dl_unbinned, s, inverse=True):
    """EB: s_nc = C^-1/2 s with 1/var set to 0 where var = 0
    (NonCenteredGibbs.py:186-194, ASIS.py:182-190); inverse=False: C^1/2 s
    (the re-centring of ASIS.py:199-203)."""
    var = H.var_from_dl(dl_unbinned)
    out = np.zeros_like(s)
    for k in range(mm.F):
        v = var[k][mm.slot_ell]
        if inverse:
            iv = np.zeros_like(v)
            iv[v != 0] = 1.0 / v[v != 0]
            out[k] = np.sqrt(iv) * s[k]
        else:
            out[k] = np.sqrt(v) * s[k]
    return out


def run_masked_mh_chain(kind, mm, model, dls_init, n_iter, draws, tol=1e-13, cr="pcg", n_gibbs=1, noise_pol0=1.0,
                        quirk=True, native=None):
    """The masked NonCenteredClsSampler.run_polarization (NonCenteredGibbs.py:529-571)
    and ASIS.run_polarization (ASIS.py:134-226) chains in the reference's
    draw order, for one chain.  cr: "pcg" or "aux_mala" (ASIS with gibbs_cr,
    its default ula=True).  native: (seed, chain) to use the device streams
    instead of numpy's (draws must then be a factory it -> NativeDraws)."""
    from . import reference_eb as RE
    binned = {s: np.array(dls_init[s], dtype=np.float64) for s in model.spectra}
    hist = {s: [binned[s].copy()] for s in model.spectra}
    accs = {s: [] for s in model.spectra}

    def dr(it):
        return draws(it) if native is not None else draws

    def mh(s_nc, start, it):
        if native is not None:
            return pixel_mh(mm, model, start, s_nc, seed=native[0], chain=native[1], iteration=it)
        u_prop, u_acc = RE.draw_mh_uniforms(model)
        return pixel_mh(mm, model, start, s_nc, u_prop=u_prop, u_accept=u_acc)

    s = None
    if kind == "asis" and cr != "pcg":
        s, _, _ = pcg_sample(mm, model.unfold(binned), dr(0), tol=tol)
    for i in range(n_iter):
        it = i + 1
        dl = model.unfold(binned)
        if kind == "noncentered":
            s, _, _ = pcg_sample(mm, dl, dr(it), tol=tol)
            binned, a = mh(noncentre(mm, dl, s), binned, it)
        else:
            if cr == "pcg":
                s, _, _ = pcg_sample(mm, dl, dr(it), tol=tol)
            else:
                s, _ = sample_dispatch(mm, dl, s, dr(it), gibbs_cr=True, overrelaxation_flag=False, ula=True,
                                       n_gibbs=n_gibbs, noise_pol0=noise_pol0)
            if native is not None:
                tmp = H.centered_cls_draw(model, H.sweep_stats(model, s, model.d_alm), seed=native[0],
                                          chain=native[1], iteration=it)
            else:
                tmp = RE.cls_centered(model, s)
            s_nc = noncentre(mm, model.unfold(tmp), s)
            binned, a = mh(s_nc, tmp, it)
            s = noncentre(mm, model.unfold(binned), s if quirk else s_nc, inverse=False)
        for sp in model.spectra:
            accs[sp].append(a[sp])
            hist[sp].append(binned[sp].copy())
    return {sp: np.array(v) for sp, v in hist.items()}, {sp: np.array(v) for sp, v in accs.items()}, s


# ----------------------------------------------------------------------------
# f4: temperature-only samplers from pixel data (TT; full sky or masked)
# ----------------------------------------------------------------------------
def tt_model(L, nside, bl, tmap, inv_noise_t):
    """the TT problem: N^-1 = (mask) / noise (ConstrainedRealization.py:22-37),
    mu = max(N^-1) + 1e-7 (:44), data term adjoint_synthesis_hp (iter 3)."""
    z = np.zeros_like(np.asarray(tmap, dtype=np.float64))
    return MaskedModel(L, nside, 1, bl, np.stack([tmap, z, z]), np.stack([inv_noise_t, z, z]), mu_eps=1e-7,
                       adj_iter=3)


def tt_fullsky_cr(mm, dl_tt, z_slot, z_pix, noncentered=False):
    """CenteredConstrainedRealization.sample_no_mask (CenteredGibbs.py:108-132) or
    NonCenteredConstrainedRealization.sample_no_mask (NonCenteredGibbs.py:22-38):
    the diagonal solve with N^-1[0] Npix/4pi for the noise precision."""
    ell = mm.slot_ell
    var = H.var_from_dl(np.atleast_2d(dl_tt))[0][ell]
    b = mm.bl[ell]
    kap = mm.inv_noise[0][0] * mm.Npix / FOURPI
    g2 = mm.second_part_grad()[0]
    y = np.sqrt(mm.inv_noise[0]) * z_pix
    f = b * mm.analysis(y[None], 3)[0] * (mm.Npix / FOURPI)
    if noncentered:
        sig = 1.0 / (1.0 + var * kap * b * b)
        return sig * (np.sqrt(var) * g2) + sig * (z_slot + np.sqrt(var) * f)
    iv = np.where((ell >= 2) & (var != 0), 1.0 / np.where(var != 0, var, 1.0), 0.0)
    sig = 1.0 / (iv + kap * b * b)
    return sig * g2 + sig * (z_slot * np.sqrt(iv) + f)


def tt_chain(kind, mm_cr, mm_mh, model, dls_init, n_iter, draws, gibbs_cr=False, tol=1e-13, native=None):
    """The reference's TT drivers in their draw order (f4 semantics):
    kind "centered": GibbsSampler.run_temperature (GibbsSampler.py:76-116);
    "noncentered": NonCenteredGibbs.run_temperature (488-527);
    "asis": ASIS.run_temperature (ASIS.py:69-131).  mm_cr: the CR problem
    (tt_model, masked or not), mm_mh the MH likelihood problem.  Full sky ->
    closed forms; masked -> PCG.  native: (seed, chain) with draws(it) ->
    NativeDraws.  Returns (history, accepts, final map)."""
    from . import reference_eb as RE
    masked = bool(np.any(mm_cr.inv_noise[0] == 0))
    nr = (mm_cr.L + 1) ** 2

    def dr(it):
        return draws(it) if native is not None else draws

    def cr_c(dl, it):
        if masked:
            d = dr(it)
            zs = d.slot_normals(1, nr, substep=SUB_PCG_S)
            zp = d.pixel_normals(1, mm_cr.Npix, maps=(0,), substep=SUB_PCG_V)
            x, _ = pcg_solve(mm_cr, dl, mm_cr.second_part_grad() + pcg_fluctuation(mm_cr, dl, zp, zs), tol)
            return x
        d = dr(it)
        zs = d.slot_normals(1, nr, substep=SUB_PCG_S)
        zp = d.pixel_normals(1, mm_cr.Npix, maps=(0,), substep=SUB_PCG_V)
        return tt_fullsky_cr(mm_cr, dl, zs[0], zp[0])[None]

    def cr_nc(dl, it):
        if masked:
            return noncentre(mm_cr, dl, cr_c(dl, it))
        d = dr(it)
        zs = d.slot_normals(1, nr, substep=SUB_PCG_S)
        zp = d.pixel_normals(1, mm_cr.Npix, maps=(0,), substep=SUB_PCG_V)
        return tt_fullsky_cr(mm_cr, dl, zs[0], zp[0], noncentered=True)[None]

    def cls(s, it):
        if native is not None:
            return H.centered_cls_draw(model, H.sweep_stats(model, s, model.d_alm), seed=native[0], chain=native[1],
                                       iteration=it)
        return RE.cls_centered(model, s)

    def mh(s_nc, start, it):
        if native is not None:
            return pixel_mh(mm_mh, model, start, s_nc, seed=native[0], chain=native[1], iteration=it)
        u_prop, u_acc = RE.draw_mh_uniforms(model)
        return pixel_mh(mm_mh, model, start, s_nc, u_prop=u_prop, u_accept=u_acc)

    binned = {"TT": np.array(dls_init["TT"], dtype=np.float64)}
    hist, accs = [], []
    s = None
    if kind in ("centered", "asis"):
        hist.append(binned["TT"].copy())
        s = cr_c(model.unfold(binned), 0)
    for i in range(n_iter):
        it = i + 1
        dl = model.unfold(binned)
        if kind == "centered":
            s = cr_c(dl, it)
            binned = cls(s, it)
        elif kind == "noncentered":
            s = cr_nc(dl, it)
            binned, a = mh(s, binned, it)
            accs.append(a["TT"])
        else:
            if gibbs_cr:
                s, _ = aux_variable(mm_cr, dl, s, 1, dr(it))
            else:
                s = cr_c(dl, it)
            tmp = cls(s, it)
            s_nc = noncentre(mm_cr, model.unfold(tmp), s)
            binned, a = mh(s_nc, tmp, it)
            accs.append(a["TT"])
            s = noncentre(mm_cr, model.unfold(binned), s_nc, inverse=False)
        hist.append(binned["TT"].copy())
    return np.array(hist), np.array(accs), s
