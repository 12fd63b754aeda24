"""numpy restatement of the harmonic-domain Gibbs hot path (TEST INFRASTRUCTURE).

Every function cites the reference line(s) it restates.  Reference paths are
relative to the upstream repository Gabriel-Ducrocq/GibbsSampler.

Conventions:
  * real m-major layout of size (L+1)^2: slots 0..L hold a_l0, then for
    m = 1..L, l = m..L the pair (sqrt2 Re a_lm, sqrt2 Im a_lm) at real slots
    2i-(L+1), 2i-(L+1)+1 with i = m(2L+1-m)/2 + l  (utils.py:49-76).
  * every real slot of multipole l carries prior variance C_l
    (utils.py:114-147), so alm2cl is S_l / (2l+1) with S_l the sum of squares
    of the slots of l.
  * fields: nfields = 1 -> (T,), 2 -> (E, B) (the reference's EE/BB runs),
    3 -> (T, E, B) with TE coupling (build-specified, reduces to the EB path
    when TT = TE = 0).
  * spectra order: nfields=1 -> [TT]; 2 -> [EE, BB]; 3 -> [TT, EE, BB, TE].
"""
import math
import numpy as np

from scipy.special import ndtri, ndtr, log_ndtr

SQRT2 = math.sqrt(2.0)
FOURPI = 4.0 * math.pi

SPECTRA = {1: ("TT",), 2: ("EE", "BB"), 3: ("TT", "EE", "BB", "TE")}
FIELDS = {1: ("T",), 2: ("E", "B"), 3: ("T", "E", "B")}


# ----------------------------------------------------------------------------
# layout helpers (utils.py:49-76, variance_expension.pyx:65-111)
# ----------------------------------------------------------------------------
def ncomplex(L):
    return (L + 1) * (L + 2) // 2


def nreal(L):
    return (L + 1) ** 2


def complex_index(L, ell, m):
    return m * (2 * L + 1 - m) // 2 + ell


def complex_ell_m(L):
    """(ell, m) of every complex m-major index (healpy Alm.getlm order)."""
    ells, ms = [], []
    for m in range(L + 1):
        ells.append(np.arange(m, L + 1))
        ms.append(np.full(L + 1 - m, m))
    return np.concatenate(ells), np.concatenate(ms)


def slot_ell(L):
    """multipole of every real slot (the index map of utils.py:121-135)."""
    ell_c, _ = complex_ell_m(L)
    out = np.empty(nreal(L), dtype=np.int64)
    out[: L + 1] = ell_c[: L + 1]
    i = np.arange(L + 1, ncomplex(L))
    out[2 * i - (L + 1)] = ell_c[i]
    out[2 * i - (L + 1) + 1] = ell_c[i]
    return out


def slot_m(L):
    _, m_c = complex_ell_m(L)
    out = np.empty(nreal(L), dtype=np.int64)
    out[: L + 1] = 0
    i = np.arange(L + 1, ncomplex(L))
    out[2 * i - (L + 1)] = m_c[i]
    out[2 * i - (L + 1) + 1] = m_c[i]
    return out


def real_to_complex(alms, L):
    """utils.py:49-60."""
    alms = np.asarray(alms, dtype=np.float64)
    m0 = alms[: L + 1] + 0j
    mp = alms[L + 1:]
    mp = (mp[::2] + 1j * mp[1::2]) / SQRT2
    return np.concatenate([m0, mp])


def complex_to_real(alms, L):
    """utils.py:63-76."""
    alms = np.asarray(alms)
    out = np.empty(nreal(L), dtype=np.float64)
    out[: L + 1] = alms[: L + 1].real
    mp = alms[L + 1:]
    out[L + 1::2] = mp.real * SQRT2
    out[L + 2::2] = mp.imag * SQRT2
    return out


def remove_monopole_dipole(alms, L):
    """variance_expension.pyx:103-111: zero slots {0, 1, L+1, L+2}."""
    out = np.array(alms, dtype=np.float64, copy=True)
    out[[0, 1, L + 1, L + 2]] = 0.0
    return out


def mask_inversion(L):
    """config.mask_inversion (cp38 bytecode): slots excluded by the rule above."""
    m = np.ones(nreal(L), dtype=bool)
    m[[0, 1, L + 1, L + 2]] = False
    return m


def dl_to_cl_factor(L):
    """GibbsSampler.py:54: 2pi/(l(l+1)), 0 at l=0."""
    ell = np.arange(L + 1, dtype=np.float64)
    f = np.zeros(L + 1)
    f[1:] = 2 * np.pi / (ell[1:] * (ell[1:] + 1))
    return f


def var_from_dl(dl):
    """Per-l variance used by generate_var_cl (utils.py:126-129):
    D_l*2*pi/(l(l+1)) for l>0, D_0 at l=0 (same operation order)."""
    dl = np.asarray(dl, dtype=np.float64)
    ell = np.arange(dl.shape[-1], dtype=np.float64)
    out = np.array(dl, copy=True)
    out[..., 1:] = dl[..., 1:] * 2 * np.pi / (ell[1:] * (ell[1:] + 1))
    return out


def generate_var_cl(dl):
    """utils.py:114-147 / variance_expension.pyx:8-33."""
    dl = np.asarray(dl, dtype=np.float64)
    L = dl.shape[-1] - 1
    return var_from_dl(dl)[..., slot_ell(L)]


def expand_per_ell(x_l):
    """Expand any per-l array to the real layout (GibbsSampler.py:73)."""
    x_l = np.asarray(x_l)
    L = x_l.shape[-1] - 1
    return x_l[..., slot_ell(L)]


def unfold_bins(binned, bins):
    """utils.py:150-162."""
    bins = np.asarray(bins)
    return np.repeat(np.asarray(binned, dtype=np.float64), bins[1:] - bins[:-1])


def gauss_beam(fwhm_rad, L):
    """healpy.gauss_beam (pol=False) as used at GibbsSampler.py:72,
    ConstrainedRealization.py:31: exp(-l(l+1) sigma^2 / 2), sigma = fwhm/sqrt(8 ln2)."""
    sigma = fwhm_rad / math.sqrt(8.0 * math.log(2.0))
    ell = np.arange(L + 1, dtype=np.float64)
    return np.exp(-0.5 * ell * (ell + 1) * sigma ** 2)


def alm2cl_real(x, y=None):
    """hp.alm2cl on the real layout: (sum over slots of l of x*y)/(2l+1)."""
    x = np.asarray(x, dtype=np.float64)
    L = int(round(math.sqrt(x.shape[-1]))) - 1
    y = x if y is None else np.asarray(y, dtype=np.float64)
    return ell_sums(x, y, L) / (2 * np.arange(L + 1) + 1)


def ell_sums(x, y, L):
    """S_l = sum over the real slots of multipole l of x*y (fp64 bincount)."""
    return np.bincount(slot_ell(L), weights=np.asarray(x) * np.asarray(y), minlength=L + 1)


# ----------------------------------------------------------------------------
# counter-based RNG (build-specified native stream; identical on the device)
# ----------------------------------------------------------------------------
PHILOX_M0 = np.uint64(0xD2511F53)
PHILOX_M1 = np.uint64(0xCD9E8D57)
PHILOX_W0 = 0x9E3779B9
PHILOX_W1 = 0xBB67AE85
MASK32 = np.uint64(0xFFFFFFFF)

TAG_CR = 1           # CR normals; c0 = complex index, c1 = field, c2 = TAG|substep<<8
TAG_GAMMA_N = 2      # gamma attempt normal; c0 = bin, c1 = spec | attempt<<8
TAG_GAMMA_U = 3      # gamma attempt uniform
TAG_GAMMA_BOOST = 4  # alpha<1 boost uniform
TAG_IW_N = 5         # Bartlett off-diagonal normal; c0 = bin
TAG_TN = 6           # truncnorm / normal proposal; c0 = bin, c1 = spec
TAG_MH_U = 7         # MH accept uniform; c0 = block, c1 = spec | attempt<<8


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Philox4x32-10 (Salmon et al. 2011) on uint32 arrays (held in uint64)."""
    c0 = np.asarray(c0, dtype=np.uint64) & MASK32
    c1 = np.asarray(c1, dtype=np.uint64) & MASK32
    c2 = np.asarray(c2, dtype=np.uint64) & MASK32
    c3 = np.asarray(c3, dtype=np.uint64) & MASK32
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    c0, c1, c2, c3 = (c.copy() for c in (c0, c1, c2, c3))
    k0 = int(k0) & 0xFFFFFFFF
    k1 = int(k1) & 0xFFFFFFFF
    for _ in range(10):
        p0 = PHILOX_M0 * c0
        p1 = PHILOX_M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK32
        n0 = hi1 ^ c1 ^ np.uint64(k0)
        n2 = hi0 ^ c3 ^ np.uint64(k1)
        c0, c1, c2, c3 = n0, lo1, n2, lo0
        k0 = (k0 + PHILOX_W0) & 0xFFFFFFFF
        k1 = (k1 + PHILOX_W1) & 0xFFFFFFFF
    return c0, c1, c2, c3


def chain_key(seed, chain):
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    return seed & 0xFFFFFFFF, ((seed >> 32) ^ int(chain)) & 0xFFFFFFFF


def u53(wa, wb):
    """uniform in (0,1) from two 32-bit words (53 bits, +half ulp)."""
    wa = np.asarray(wa, dtype=np.uint64)
    wb = np.asarray(wb, dtype=np.uint64)
    k = (wa >> np.uint64(5)).astype(np.float64) * 67108864.0 + (wb >> np.uint64(6)).astype(np.float64)
    return (k + 0.5) * (1.0 / 9007199254740992.0)


def box_muller(w0, w1, w2, w3):
    u1 = u53(w0, w1)
    u2 = u53(w2, w3)
    r = np.sqrt(-2.0 * np.log(u1))
    th = 2.0 * np.pi * u2
    return r * np.cos(th), r * np.sin(th)


def cr_normals(seed, chain, iteration, substep, field, L):
    """Native CR normal stream for one (chain, field): z in the real layout."""
    k0, k1 = chain_key(seed, chain)
    i = np.arange(ncomplex(L), dtype=np.uint64)
    w = philox4x32_10(i, field, TAG_CR | (substep << 8), iteration, k0, k1)
    z0, z1 = box_muller(*w)
    z = np.empty(nreal(L))
    z[: L + 1] = z0[: L + 1]
    ii = np.arange(L + 1, ncomplex(L))
    z[2 * ii - (L + 1)] = z0[L + 1:]
    z[2 * ii - (L + 1) + 1] = z1[L + 1:]
    return z


def _normal1(k0, k1, c0, c1, c2, c3):
    w = philox4x32_10(c0, c1, c2, c3, k0, k1)
    z0, _ = box_muller(*w)
    return float(z0)


def _uniform1(k0, k1, c0, c1, c2, c3):
    w = philox4x32_10(c0, c1, c2, c3, k0, k1)
    return float(u53(w[0], w[1]))


def gamma_native(alpha, k0, k1, b, spec, iteration, sub=0):
    """Marsaglia-Tsang Gamma(alpha, 1) on the counter stream (alpha>0).
    Attempt j uses counters (b, spec | j<<8, TAG_GAMMA_N|sub<<8, it) and
    (b, spec | j<<8, TAG_GAMMA_U|sub<<8, it).  alpha < 1 uses the boost
    G(alpha) = G(alpha+1) * U^(1/alpha)."""
    a = alpha if alpha >= 1.0 else alpha + 1.0
    d = a - 1.0 / 3.0
    c = 1.0 / math.sqrt(9.0 * d)
    j = 0
    while True:
        cc = spec | (j << 8)
        x = _normal1(k0, k1, b, cc, TAG_GAMMA_N | (sub << 8), iteration)
        u = _uniform1(k0, k1, b, cc, TAG_GAMMA_U | (sub << 8), iteration)
        j += 1
        t = 1.0 + c * x
        if t <= 0.0:
            continue
        v = t * t * t
        if u < 1.0 - 0.0331 * (x * x) * (x * x) or math.log(u) < 0.5 * x * x + d * (1.0 - v + math.log(v)):
            g = d * v
            break
    if alpha < 1.0:
        ub = _uniform1(k0, k1, b, spec, TAG_GAMMA_BOOST | (sub << 8), iteration)
        g = g * math.exp(math.log(ub) / alpha)
    return g


# ----------------------------------------------------------------------------
# model description
# ----------------------------------------------------------------------------
class Model:
    """Static model of one Gibbs problem (SURVEY.md 8d, config.py:19-90).

    kappa_X = Npix / (4 pi sigma_X^2) is the per-field harmonic noise precision
    (CenteredGibbs.py:336,340; NonCenteredGibbs.py:150,162)."""

    def __init__(self, L, nside, nfields, bl, noise_var, bins, blocks=None,
                 proposal_variances=None, d_alm=None):
        self.L = int(L)
        self.nside = int(nside)
        self.Npix = 12 * self.nside ** 2
        self.nfields = int(nfields)
        self.spectra = SPECTRA[self.nfields]
        self.fields = FIELDS[self.nfields]
        self.bl = np.asarray(bl, dtype=np.float64)
        self.noise_var = [float(v) for v in noise_var]           # per field
        self.kappa = [self.Npix / (4 * np.pi * v) for v in self.noise_var]
        self.bins = {s: np.asarray(bins[s], dtype=np.int64) for s in self.spectra}
        self.blocks = None if blocks is None else {s: np.asarray(blocks[s], dtype=np.int64) for s in self.spectra}
        self.proposal_variances = None if proposal_variances is None else \
            {s: np.asarray(proposal_variances[s], dtype=np.float64) for s in self.spectra}
        self.d_alm = None if d_alm is None else np.asarray(d_alm, dtype=np.float64)   # [F, (L+1)^2]

    def nbins(self, spec):
        return len(self.bins[spec]) - 1

    def unfold(self, dl_binned):
        """dict spec -> binned D  ->  [nspec, L+1] unbinned D."""
        return np.stack([unfold_bins(dl_binned[s], self.bins[s]) for s in self.spectra])

    def ell_to_bin(self, spec):
        b = self.bins[spec]
        out = np.full(self.L + 1, -1, dtype=np.int64)
        for k in range(len(b) - 1):
            out[b[k]:b[k + 1]] = k
        return out


# ----------------------------------------------------------------------------
# per-l block algebra
# ----------------------------------------------------------------------------
def _spec_index(model, name):
    return model.spectra.index(name) if name in model.spectra else None


def cov_blocks(model, dl_unbinned):
    """Per-l signal covariance C_l (3x3 for TEB, diag otherwise) in C units
    (generate_var_cl semantics: l=0 keeps D_0)."""
    var = var_from_dl(dl_unbinned)            # [nspec, L+1]
    F = model.nfields
    C = np.zeros((model.L + 1, F, F))
    if F == 1:
        C[:, 0, 0] = var[0]
    elif F == 2:
        C[:, 0, 0] = var[0]
        C[:, 1, 1] = var[1]
    else:
        C[:, 0, 0] = var[0]
        C[:, 1, 1] = var[1]
        C[:, 2, 2] = var[2]
        C[:, 0, 1] = C[:, 1, 0] = var[3]
    return C


def _pinv_te_block(a, b, c):
    """Zero-variance rule generalised to the 2x2 TE block
    [[a, c], [c, b]]: a component with zero auto-variance gets zero prior
    precision (and its cross term is ignored)."""
    if a != 0.0 and b != 0.0:
        det = a * b - c * c
        return b / det, a / det, -c / det
    ia = 1.0 / a if a != 0.0 else 0.0
    ib = 1.0 / b if b != 0.0 else 0.0
    return ia, ib, 0.0


def inv_var(v):
    """inv[v != 0] = 1/v, 0 elsewhere (CenteredGibbs.py:330-334)."""
    v = np.asarray(v, dtype=np.float64)
    out = np.zeros_like(v)
    nz = v != 0
    out[nz] = 1.0 / v[nz]
    return out


def centered_params(model, dl_unbinned):
    """Per-l (M, Lchol) of the centered full-sky CR: s = M d + Lchol z.

    EB/T: exactly CenteredGibbs.py:324-351 per slot (sigma, r = kappa b d).
    TEB: Q = C^+ + diag(b^2 kappa), Sigma = Q^-1, M = Sigma diag(b kappa)."""
    L, F = model.L, model.nfields
    bl = model.bl
    var = var_from_dl(dl_unbinned)
    M = np.zeros((L + 1, F, F))
    Lc = np.zeros((L + 1, F, F))
    if F != 3:
        for f in range(F):
            kap = model.kappa[f]
            sig = 1.0 / ((model.Npix / (model.noise_var[f] * 4 * np.pi)) * bl ** 2 + inv_var(var[f]))
            M[:, f, f] = sig * ((model.Npix * (1.0 / model.noise_var[f]) / (4 * np.pi)) * bl)
            Lc[:, f, f] = np.sqrt(sig)
        return M, Lc
    C = cov_blocks(model, dl_unbinned)
    for ell in range(L + 1):
        p = [bl[ell] ** 2 * k for k in model.kappa]
        it, ie, ite = _pinv_te_block(C[ell, 0, 0], C[ell, 1, 1], C[ell, 0, 1])
        q00, q11, q01 = it + p[0], ie + p[1], ite
        det = q00 * q11 - q01 * q01
        s00, s11, s01 = q11 / det, q00 / det, -q01 / det
        ib = 1.0 / C[ell, 2, 2] if C[ell, 2, 2] != 0.0 else 0.0
        s22 = 1.0 / (ib + p[2])
        bk = [bl[ell] * k for k in model.kappa]
        M[ell, 0, 0], M[ell, 0, 1] = s00 * bk[0], s01 * bk[1]
        M[ell, 1, 0], M[ell, 1, 1] = s01 * bk[0], s11 * bk[1]
        M[ell, 2, 2] = s22 * bk[2]
        l00 = math.sqrt(s00)
        l10 = s01 / l00
        l11 = math.sqrt(max(s11 - l10 * l10, 0.0))
        Lc[ell, 0, 0], Lc[ell, 1, 0], Lc[ell, 1, 1] = l00, l10, l11
        Lc[ell, 2, 2] = math.sqrt(s22)
    return M, Lc


def cov_chol(model, dl_unbinned):
    """Cholesky factor of C_l with the zero-variance rule (non-centering map;
    EB: sqrt(var), NonCenteredGibbs.py:165-166)."""
    C = cov_blocks(model, dl_unbinned)
    F = model.nfields
    A = np.zeros_like(C)
    if F != 3:
        for f in range(F):
            A[:, f, f] = np.sqrt(C[:, f, f])
        return A
    for ell in range(model.L + 1):
        a, b, c = C[ell, 0, 0], C[ell, 1, 1], C[ell, 0, 1]
        if a != 0.0:
            l00 = math.sqrt(a)
            l10 = c / l00
            l11 = math.sqrt(max(b - l10 * l10, 0.0))
        else:
            l00, l10, l11 = 0.0, 0.0, math.sqrt(b)
        A[ell, 0, 0], A[ell, 1, 0], A[ell, 1, 1] = l00, l10, l11
        A[ell, 2, 2] = math.sqrt(C[ell, 2, 2])
    return A


def chol_pinv(A):
    """Pseudo-inverse of the per-l lower-triangular factor (zero rule):
    EB: sqrt(inv_var) (ASIS.py:185-189)."""
    F = A.shape[-1]
    out = np.zeros_like(A)
    for ell in range(A.shape[0]):
        if F != 3:
            for f in range(F):
                out[ell, f, f] = 1.0 / A[ell, f, f] if A[ell, f, f] != 0.0 else 0.0
            continue
        l00, l10, l11 = A[ell, 0, 0], A[ell, 1, 0], A[ell, 1, 1]
        i00 = 1.0 / l00 if l00 != 0.0 else 0.0
        i11 = 1.0 / l11 if l11 != 0.0 else 0.0
        out[ell, 0, 0] = i00
        out[ell, 1, 1] = i11
        out[ell, 1, 0] = -l10 * i00 * i11
        out[ell, 2, 2] = 1.0 / A[ell, 2, 2] if A[ell, 2, 2] != 0.0 else 0.0
    return out


def noncentered_params(model, dl_unbinned):
    """Per-l (M, Lchol) of the non-centered full-sky CR (all_sph):
    EB: NonCenteredGibbs.py:141-174 -- sigma = 1/(1 + kappa b^2 C),
    mean = sigma sqrt(C) b kappa d.
    TEB: Q = I + A^T diag(b^2 kappa) A, A = chol(C); M = Q^-1 A^T diag(b kappa)."""
    L, F = model.L, model.nfields
    bl = model.bl
    var = var_from_dl(dl_unbinned)
    M = np.zeros((L + 1, F, F))
    Lc = np.zeros((L + 1, F, F))
    if F != 3:
        for f in range(F):
            inv_n = 1.0 / model.noise_var[f]
            sig = 1.0 / (1.0 + inv_n * bl ** 2 * var[f] * model.Npix / (4 * np.pi))
            M[:, f, f] = sig * (np.sqrt(var[f]) * bl * (model.Npix * inv_n / (4 * np.pi)))
            Lc[:, f, f] = np.sqrt(sig)
        return M, Lc
    A = cov_chol(model, dl_unbinned)
    for ell in range(L + 1):
        P = np.diag([bl[ell] ** 2 * k for k in model.kappa])
        Q = np.eye(3) + A[ell].T @ P @ A[ell]
        S = np.linalg.inv(Q)
        S = 0.5 * (S + S.T)
        M[ell] = S @ A[ell].T @ np.diag([bl[ell] * k for k in model.kappa])
        Lc[ell] = np.linalg.cholesky(S)
    return M, Lc


def cr_apply(model, M, Lc, d, z):
    """s = M_l d + Lchol_l z slot by slot.  d, z: [F, (L+1)^2] -> s [F, (L+1)^2]."""
    ell = slot_ell(model.L)
    F = model.nfields
    s = np.zeros_like(z)
    for f in range(F):
        for g in range(F):
            if np.any(M[:, f, g] != 0):
                s[f] += M[ell, f, g] * d[g]
    for f in range(F):
        for g in range(F):
            if np.any(Lc[:, f, g] != 0):
                s[f] += Lc[ell, f, g] * z[g]
    return s


def cr_apply_eb_reference(model, M, Lc, d, z):
    """EB/T with the reference's exact operation order: mean + z*sqrt(sigma)."""
    ell = slot_ell(model.L)
    return np.stack([M[ell, f, f] * d[f] + z[f] * Lc[ell, f, f] for f in range(model.nfields)])


def sweep_stats(model, s, d):
    """Per-l sufficient statistics accumulated by the fused CR sweep.
    Returns dict with 'ss' [F,F,L+1] (sum s_X s_Y) and 'ds' [F,F,L+1]
    (sum d_X s_Y) -- only the couplings present in the model are non-zero."""
    L, F = model.L, model.nfields
    ss = np.zeros((F, F, L + 1))
    ds = np.zeros((F, F, L + 1))
    for f in range(F):
        for g in range(F):
            if F == 3 and (f == 2) != (g == 2):
                continue
            if F != 3 and f != g:
                continue
            ss[f, g] = ell_sums(s[f], s[g], L)
            ds[f, g] = ell_sums(d[f], s[g], L)
    return {"ss": ss, "ds": ds}


def centered_betas(model, ss):
    """beta_l = (2l+1) l(l+1) Chat_l / (4 pi) = l(l+1) S_l/(4 pi)
    (CenteredGibbs.py:61-66) for every spectrum."""
    L = model.L
    ell = np.arange(L + 1, dtype=np.float64)
    chat = {}
    F = model.nfields
    if F == 1:
        chat["TT"] = ss[0, 0]
    elif F == 2:
        chat["EE"], chat["BB"] = ss[0, 0], ss[1, 1]
    else:
        chat["TT"], chat["EE"], chat["BB"], chat["TE"] = ss[0, 0], ss[1, 1], ss[2, 2], ss[0, 1]
    return {k: v / (2 * ell + 1) for k, v in chat.items()}


def invgamma_params(model, spec, chat):
    """Per-bin (alpha, beta) of CenteredGibbs.py:62-76 (alpha_0 := 1)."""
    L = model.L
    ell = np.arange(L + 1, dtype=np.float64)
    betas = (2 * ell + 1) * ell * (ell + 1) * (chat / (4 * np.pi))
    expo = (2 * ell + 1) / 2
    b = model.bins[spec]
    alphas, bs = [], []
    for i in range(len(b) - 1):
        bs.append(np.sum(betas[b[i]:b[i + 1]]))
        alphas.append(np.sum(expo[b[i]:b[i + 1]]) - 1)
    alphas[0] = 1
    return np.array(alphas, dtype=np.float64), np.array(bs, dtype=np.float64)


def centered_cls_draw(model, stats, variates=None, seed=0, chain=0, iteration=0):
    """C_l step of the centered sampler.

    EB/T: PolarizedCenteredClsSampler.sample (CenteredGibbs.py:54-93): one
    inverse-Gamma vector per spectrum, D = beta * X, D[:2] = 0.
    ``variates[spec]`` = the invgamma.rvs(alpha) vector (replay); else native.
    TEB: TT/EE/TE share bins and are drawn by a per-bin 2x2 inverse-Wishart
    IW(nu_b, Psi_b), nu_b = sum(2l+1) - 3, Psi_b = sum l(l+1)/(2pi) S_l;
    BB stays inverse-Gamma (build spec; p=1 reduces to the above)."""
    chat = centered_betas(model, stats["ss"])
    k0, k1 = chain_key(seed, chain)
    out = {}
    ig_specs = [s for s in model.spectra if not (model.nfields == 3 and s in ("TT", "EE", "TE"))]
    for si, spec in enumerate(model.spectra):
        if spec not in ig_specs:
            continue
        alphas, betas = invgamma_params(model, spec, chat[spec])
        if variates is not None:
            X = np.asarray(variates[spec], dtype=np.float64)
        else:
            X = np.array([0.0 if b < 2 else 1.0 / gamma_native(alphas[b], k0, k1, b, si, iteration)
                          for b in range(len(alphas))])
        dl = betas * X
        dl[:2] = 0.0
        out[spec] = dl
    if model.nfields == 3:
        out.update(_iw_te_draw(model, stats["ss"], k0, k1, iteration))
    return {s: out[s] for s in model.spectra}


def iw_bin_params(model, ss):
    """Per-bin (nu, Psi) for the TT/EE/TE inverse-Wishart (D units)."""
    L = model.L
    ell = np.arange(L + 1, dtype=np.float64)
    w = ell * (ell + 1) / (2 * np.pi)
    b = model.bins["TT"]
    nb = len(b) - 1
    nu = np.zeros(nb)
    psi = np.zeros((nb, 3))   # TT, EE, TE
    for i in range(nb):
        sl = slice(b[i], b[i + 1])
        nu[i] = np.sum(2 * ell[sl] + 1) - 3
        psi[i, 0] = np.sum(w[sl] * ss[0, 0, sl])
        psi[i, 1] = np.sum(w[sl] * ss[1, 1, sl])
        psi[i, 2] = np.sum(w[sl] * ss[0, 1, sl])
    return nu, psi


def _iw_te_draw(model, ss, k0, k1, iteration):
    """Bartlett draw of W ~ Wishart(nu, Psi^-1), D = W^-1, per bin b >= 2."""
    nu, psi = iw_bin_params(model, ss)
    nb = len(nu)
    tt, ee, te = np.zeros(nb), np.zeros(nb), np.zeros(nb)
    for b in range(2, nb):
        a, d_, c = psi[b]
        det = a * d_ - c * c
        # S = Psi^-1 = [[d, -c], [-c, a]] / det ; L = chol(S)
        s00, s11, s01 = d_ / det, a / det, -c / det
        l00 = math.sqrt(s00)
        l10 = s01 / l00
        l11 = math.sqrt(s11 - l10 * l10)
        c1 = math.sqrt(2.0 * gamma_native(0.5 * nu[b], k0, k1, b, 16, iteration))
        c2 = math.sqrt(2.0 * gamma_native(0.5 * (nu[b] - 1.0), k0, k1, b, 17, iteration))
        n = _normal1(k0, k1, b, 0, TAG_IW_N, iteration)
        # B = L A, A = [[c1, 0], [n, c2]]
        b00 = l00 * c1
        b10 = l10 * c1 + l11 * n
        b11 = l11 * c2
        # W = B B^T ; D = W^-1
        w00 = b00 * b00
        w01 = b00 * b10
        w11 = b10 * b10 + b11 * b11
        wd = w00 * w11 - w01 * w01
        tt[b], ee[b], te[b] = w11 / wd, w00 / wd, -w01 / wd
    return {"TT": tt, "EE": ee, "TE": te}


# ----------------------------------------------------------------------------
# non-centered Metropolis-within-Gibbs (NonCenteredGibbs.py:252-445)
# ----------------------------------------------------------------------------
def truncnorm_ppf_std(q, a):
    """Standard normal truncated to [a, inf), a <= 0 (scipy truncnorm._ppf
    'case_left': Phi(x) = Phi(a) + q Phi(-a)), upper tail without cancellation."""
    q = np.asarray(q, dtype=np.float64)
    a = np.asarray(a, dtype=np.float64)
    pa = ndtr(a)
    pma = ndtr(-a)
    plo = pa + q * pma
    phi = (1.0 - q) * pma
    return np.where(plo < 0.5, ndtri(plo), -ndtri(phi))


def truncnorm_log_ratio(old, prop, sd):
    """q(old|prop) - q(prop|old) of the truncated-normal proposal
    (NonCenteredGibbs.py:313-330,410-413); the Gaussian kernels cancel."""
    return log_ndtr(np.asarray(old) / sd) - log_ndtr(np.asarray(prop) / sd)


def nc_loglik_terms(model, dl_unbinned, stats, spec_only=None):
    """f_l = -1/2 sum_X kappa_X sum_slots (d_X - b (A s)_X)^2 without the
    constant S_dd term (NonCenteredGibbs.py:357-377 decomposed per l)."""
    L, F = model.L, model.nfields
    bl = model.bl
    A = cov_chol(model, dl_unbinned)
    ss, ds = stats["ss"], stats["ds"]
    f = np.zeros(L + 1)
    for X in range(F):
        kap = model.kappa[X]
        lin = np.zeros(L + 1)
        quad = np.zeros(L + 1)
        for Y in range(F):
            aXY = A[:, X, Y]
            if not np.any(aXY):
                continue
            lin += aXY * ds[X, Y]
            for Z in range(F):
                aXZ = A[:, X, Z]
                if not np.any(aXZ):
                    continue
                quad += aXY * aXZ * ss[Y, Z]
        f += -0.5 * kap * (-2.0 * bl * lin + bl ** 2 * quad)
    return f


def _psd_ok(model, dl_unbinned, ells):
    if model.nfields != 3:
        return True
    var = var_from_dl(dl_unbinned)
    tt, ee, te = var[0, ells], var[1, ells], var[3, ells]
    ok = np.where((tt == 0) & (te == 0), ee >= 0, (tt > 0) & (ee > 0) & (tt * ee - te * te > 0))
    return bool(np.all(ok))


def nc_mh(model, dl_binned_old, stats, seed=0, chain=0, iteration=0,
          u_prop=None, u_accept=None, n_iter=1, loglik=None):
    """One Metropolis-within-Gibbs sweep (PolarizationNonCenteredClsSampler.sample).

    Replay: u_prop[spec] are the truncnorm uniforms (bins >= 2, scipy draws
    them as uniform(size)), u_accept is the flat list of accept uniforms in
    block order.  Native: counter streams TAG_TN / TAG_MH_U.
    Blocks are evaluated with per-l likelihood terms; spectra in model order,
    except EB where the reference order EE, BB is also the model order.
    TEB order: EE, BB, TT, TE (the reference's EE, BB first)."""
    k0, k1 = chain_key(seed, chain)
    cur = {s: np.array(dl_binned_old[s], dtype=np.float64) for s in model.spectra}
    prop = {}
    logr = {}
    order = list(model.spectra) if model.nfields != 3 else ["EE", "BB", "TT", "TE"]
    for s in order:
        si = model.spectra.index(s)
        pv = model.proposal_variances[s]
        sd = np.sqrt(pv)
        nb = len(cur[s])
        if s == "TE":
            if u_prop is not None:
                y = ndtri(np.asarray(u_prop[s]))
            else:
                y = np.array([_normal1(k0, k1, b, si, TAG_TN, iteration) for b in range(2, nb)])
            p = cur[s][2:] + sd * y
            lr = np.zeros(nb - 2)
        else:
            a = -cur[s][2:] / sd
            if u_prop is not None:
                q = np.asarray(u_prop[s])
            else:
                q = np.array([_uniform1(k0, k1, b, si, TAG_TN, iteration) for b in range(2, nb)])
            p = cur[s][2:] + sd * truncnorm_ppf_std(q, a)
            lr = truncnorm_log_ratio(cur[s][2:], p, sd)
        prop[s] = np.concatenate([np.zeros(2), p])
        logr[s] = np.concatenate([np.zeros(2), lr])
    accept = {s: [] for s in model.spectra}
    ui = 0
    for s in order:
        si = model.spectra.index(s)
        blocks = model.blocks[s]
        nb = len(cur[s])
        for bi in range(len(blocks) - 1):
            lo, hi = int(blocks[bi]), min(int(blocks[bi + 1]), nb)
            edges = model.bins[s]
            ells = np.arange(edges[lo], edges[hi]) if hi > lo else np.arange(0)
            for it in range(n_iter):
                new = {k: v.copy() for k, v in cur.items()}
                new[s][lo:hi] = prop[s][lo:hi]
                lr_all = float(np.sum(logr[s][lo:hi]))
                un_old = model.unfold(cur)
                un_new = model.unfold(new)
                if loglik is not None:
                    # pixel-domain likelihood (NonCenteredGibbs.py:333-355,380-399):
                    # new_lik - old_lik of the whole map
                    log_r = (loglik(un_new) - loglik(un_old)) + lr_all
                elif _psd_ok(model, un_new, ells):
                    f_old = nc_loglik_terms(model, un_old, stats)
                    f_new = nc_loglik_terms(model, un_new, stats)
                    dlik = float(np.sum(f_new[ells] - f_old[ells]))
                    log_r = dlik + lr_all
                else:
                    log_r = -np.inf
                if u_accept is not None:
                    u = float(u_accept[ui])
                else:
                    u = _uniform1(k0, k1, bi, si | (it << 8), TAG_MH_U, iteration)
                ui += 1
                if math.log(u) < log_r:
                    cur = new
                    accept[s].append(1)
                else:
                    accept[s].append(0)
    return cur, accept


def transform_stats(stats, T):
    """Stats of s' = T_l s (per-l linear map): ss' = T ss T^T, ds' = ds T^T."""
    ss, ds = stats["ss"], stats["ds"]
    F = ss.shape[0]
    ssf = ss.copy()
    dsf = ds.copy()
    # symmetrise ss (only the lower couplings may be stored)
    for f in range(F):
        for g in range(F):
            if g > f:
                ssf[f, g] = np.where(ss[f, g] != 0, ss[f, g], ss[g, f])
                ssf[g, f] = ssf[f, g]
    Tt = np.transpose(T, (1, 2, 0))       # [F, F, L+1]
    ss_new = np.einsum("ial,ajl,bjl->ibl", Tt, ssf, Tt)
    ds_new = np.einsum("xal,bal->xbl", dsf, Tt)
    return {"ss": ss_new, "ds": ds_new}
