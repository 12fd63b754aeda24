"""Reference-order EB drivers on numpy's legacy global RNG (TEST INFRASTRUCTURE).

These replay the reference's full-sky, isotropic-noise Gibbs samplers with the
exact draw order of numpy's global MT19937 stream, so that
results can be compared with golden vectors produced by the reference itself
(tests/golden, tools/gen_golden.py) and with the HIP path in replay mode.

  * centered CR (CenteredGibbs.py:317-353): z_E, z_B   (normal, (L+1)^2 each)
  * non-centered CR all_sph (NonCenteredGibbs.py:134-176): z_E, z_B
  * centered C_l draw (CenteredGibbs.py:54-93): invgamma.rvs EE, then BB
  * NC MH (NonCenteredGibbs.py:401-445): truncnorm uniforms EE (bins>=2),
    BB, then one uniform per (block, attempt) in order EE blocks, BB blocks.
"""
import numpy as np
from scipy.stats import invgamma

from . import harmonic as H


def draw_cr_normals(model):
    n = H.nreal(model.L)
    return np.stack([np.random.normal(size=n) for _ in range(model.nfields)])


def draw_invgamma(model, spec):
    alphas = _alphas(model, spec)
    return invgamma.rvs(a=alphas)


def _alphas(model, spec):
    ell = np.arange(model.L + 1, dtype=np.float64)
    expo = (2 * ell + 1) / 2
    b = model.bins[spec]
    a = np.array([np.sum(expo[b[i]:b[i + 1]]) - 1 for i in range(len(b) - 1)])
    a[0] = 1
    return a


def draw_mh_uniforms(model, n_iter=1):
    u_prop = {s: np.random.uniform(size=model.nbins(s) - 2) for s in model.spectra}
    nacc = 0
    for s in model.spectra:
        bl = model.blocks[s]
        nacc += (len(bl) - 1) * n_iter
    u_acc = np.random.uniform(size=nacc)
    return u_prop, u_acc


def cr_centered(model, dl_unbinned):
    M, Lc = H.centered_params(model, dl_unbinned)
    z = draw_cr_normals(model)
    return H.cr_apply_eb_reference(model, M, Lc, model.d_alm, z)


def cr_noncentered(model, dl_unbinned):
    M, Lc = H.noncentered_params(model, dl_unbinned)
    z = draw_cr_normals(model)
    return H.cr_apply_eb_reference(model, M, Lc, model.d_alm, z)


def cls_centered(model, s):
    stats = H.sweep_stats(model, s, model.d_alm)
    var = {sp: draw_invgamma(model, sp) for sp in model.spectra}
    return H.centered_cls_draw(model, stats, variates=var)


def nc_mh(model, s_nc, dl_binned, n_iter=1):
    u_prop, u_acc = draw_mh_uniforms(model, n_iter)
    stats = H.sweep_stats(model, s_nc, model.d_alm)
    return H.nc_mh(model, dl_binned, stats, u_prop=u_prop, u_accept=u_acc, n_iter=n_iter)


def run_centered(model, dls_init, n_iter):
    """GibbsSampler.run_polarization (GibbsSampler.py:118-180) with the
    full-sky closed-form CR; init CR (ula=True, GibbsSampler.py:41,136-138)."""
    h = {s: [np.asarray(dls_init[s], dtype=np.float64)] for s in model.spectra}
    binned = {s: np.asarray(dls_init[s], dtype=np.float64) for s in model.spectra}
    skymap = cr_centered(model, model.unfold(binned))
    for _ in range(n_iter):
        skymap = cr_centered(model, model.unfold(binned))
        binned = cls_centered(model, skymap)
        for s in model.spectra:
            h[s].append(binned[s])
    return {s: np.array(v) for s, v in h.items()}, skymap


def run_noncentered(model, dls_init, n_iter, n_iter_metropolis=1):
    """NonCenteredGibbs.run_polarization (NonCenteredGibbs.py:529-571), all_sph."""
    h = {s: [np.asarray(dls_init[s], dtype=np.float64)] for s in model.spectra}
    acc = {s: [] for s in model.spectra}
    binned = {s: np.asarray(dls_init[s], dtype=np.float64) for s in model.spectra}
    s_nc = None
    for _ in range(n_iter):
        s_nc = cr_noncentered(model, model.unfold(binned))
        binned, a = nc_mh(model, s_nc, binned, n_iter_metropolis)
        for s in model.spectra:
            h[s].append(binned[s])
            acc[s].append(a[s])
    return {s: np.array(v) for s, v in h.items()}, {s: np.array(v) for s, v in acc.items()}, s_nc


def run_asis(model, dls_init, n_iter, n_iter_metropolis=1, quirk_recentre=True):
    """ASIS.run_polarization (ASIS.py:134-226) with the full-sky CR; the
    re-centring multiplies the centered map (ASIS.py:203) when quirk_recentre."""
    h = {s: [] for s in model.spectra}
    acc = {s: [] for s in model.spectra}
    binned = {s: np.asarray(dls_init[s], dtype=np.float64) for s in model.spectra}
    skymap = None
    for _ in range(n_iter):
        skymap = cr_centered(model, model.unfold(binned))
        tmp = cls_centered(model, skymap)
        A_tmp = H.cov_chol(model, model.unfold(tmp))
        Ainv = H.chol_pinv(A_tmp)
        ell = H.slot_ell(model.L)
        s_nc = np.stack([Ainv[ell, f, f] * skymap[f] for f in range(model.nfields)])
        binned, a = nc_mh(model, s_nc, tmp, n_iter_metropolis)
        A_new = H.cov_chol(model, model.unfold(binned))
        src = skymap if quirk_recentre else s_nc
        skymap = np.stack([A_new[ell, f, f] * src[f] for f in range(model.nfields)])
        for s in model.spectra:
            h[s].append(binned[s])
            acc[s].append(a[s])
    return {s: np.array(v) for s, v in h.items()}, {s: np.array(v) for s, v in acc.items()}, skymap
