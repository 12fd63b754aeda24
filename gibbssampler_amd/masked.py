"""Masked (pixel-domain) constrained realisation on the GPU: the reference's
PolarizedCenteredConstrainedRealization masked samplers (CenteredGibbs.py:241-850).

``MaskedCR`` keeps the reference's method names and return conventions
(dict of real-layout arrays, accept flag) so a caller of the reference finds
the same surface:

  sample_gibbs_change_variable(all_dls, s_old)   a9   CenteredGibbs.py:676-729
  overrelaxation_sampler(all_dls, s_old)         a10  CenteredGibbs.py:733-825
  sample_mala(all_dls, s_old)                    a11  CenteredGibbs.py:560-603
  compute_gradient_mala(all_dls, s_old)               CenteredGibbs.py:494-520
  sample_mask(all_dls)                           f1   CenteredGibbs.py:448-491 (PCG)
  sample(all_dls, s_old=None)                    a12  CenteredGibbs.py:828-850

All arithmetic runs in libgibbs_hip.so (gs_masked_cr + gs_sht); this module
only moves arrays and, in replay mode, draws numpy's legacy global stream in
the reference's order (A.5 of SURVEY.md) so results match the reference for
the same ``np.random.seed``.  There is no CPU fallback.
"""
import ctypes
import time

import numpy as np
import torch

from . import _capi

FIELDS = {1: ("TT",), 2: ("EE", "BB"), 3: ("TT", "EE", "BB")}
SPECS = {1: ("TT",), 2: ("EE", "BB"), 3: ("TT", "EE", "BB", "TE")}


class MaskedCR:
    """pix_map: dict with "Q", "U" (and "T" for nfields = 3) pixel maps, or for
    nfields = 1 (temperature) the T map (array or dict with "T");
    noise_temp / noise_pol: per-pixel noise variances (arrays or scalars);
    mask: per-pixel mask multiplying N^-1 (CenteredGibbs.py:266-274) or None.
    Temperature contexts use the TT constants of ConstrainedRealization.py:44
    (mu = max(N^-1) + 1e-7) and healpy's default iter = 3 for the data term
    and the aux s | v analysis (utils.adjoint_synthesis_hp, CenteredGibbs.py:208)."""

    def __init__(self, pix_map, noise_temp, noise_pol, bl, lmax, nside, mask=None, nfields=2, gibbs_cr=True,
                 n_gibbs=1, alpha=-0.995, overrelaxation=False, ula=False, tau=0.02, rng="replay", seed=0, chain=0,
                 device="cuda", pcg_accuracy=1.0e-5, pcg_maxiter=4000, rj=False):
        if nfields not in (1, 2, 3):
            raise ValueError("nfields must be 1 (T), 2 (EB, the reference) or 3 (TEB)")
        self.lib = _capi.load()
        self.L, self.nside, self.F = int(lmax), int(nside), int(nfields)
        self.Npix = 12 * self.nside ** 2
        self.NR = (self.L + 1) ** 2
        self.gibbs_cr, self.overrelaxation, self.ula = bool(gibbs_cr), bool(overrelaxation), bool(ula)
        # rj: the RJPO branch of the ladder (CenteredGibbs.py:837-838, disabled at
        # HEAD by "and False"; sample_mask_rj itself is always callable)
        self.rj = bool(rj)
        self.n_gibbs, self.alpha, self.tau = int(n_gibbs), float(alpha), float(tau)
        self.pcg_accuracy, self.pcg_maxiter = float(pcg_accuracy), int(pcg_maxiter)   # CenteredGibbs.py:279-283
        self.pcg_iterations = []
        self.pcg_syncs = []
        if rng not in ("replay", "native"):
            raise ValueError(rng)
        self.rng, self.seed, self.chain = rng, int(seed), int(chain)
        self.iteration = 0
        self.device = device
        npol = np.broadcast_to(np.asarray(noise_pol, dtype=np.float64), (self.Npix,))
        ntemp = np.broadcast_to(np.asarray(noise_temp, dtype=np.float64), (self.Npix,))
        m = np.ones(self.Npix) if mask is None else np.asarray(mask, dtype=np.float64)
        inv = np.stack([m / ntemp, m / npol, m / npol])
        zero = np.zeros(self.Npix)
        if self.F == 1:
            t = pix_map["T"] if isinstance(pix_map, dict) else pix_map
            maps = np.stack([np.asarray(t, dtype=np.float64), zero, zero])
        else:
            maps = np.stack([np.asarray(pix_map.get("T", zero), dtype=np.float64),
                             np.asarray(pix_map["Q"], dtype=np.float64), np.asarray(pix_map["U"], dtype=np.float64)])
        self._maps = torch.from_numpy(np.ascontiguousarray(maps)).to(device)
        self._inv = torch.from_numpy(np.ascontiguousarray(inv)).to(device)
        self.bl = np.ascontiguousarray(np.asarray(bl, dtype=np.float64)[: self.L + 1])
        desc = _capi.GsMaskedDesc()
        desc.lmax, desc.nside, desc.nfields = self.L, self.nside, self.F
        desc.bl = self.bl.ctypes.data_as(_capi.c_double_p)
        desc.n_gibbs, desc.alpha, desc.tau, desc.noise_pol0 = self.n_gibbs, self.alpha, self.tau, float(npol[0])
        desc.mu_eps = 1e-7 if self.F == 1 else 1e-14
        desc.adj_iter = 3 if self.F == 1 else 0
        h = ctypes.c_void_p()
        _capi.check(self.lib.gs_masked_create(ctypes.byref(desc), _capi.ptr(self._maps), _capi.ptr(self._inv),
                                              ctypes.byref(h)), "gs_masked_create")
        self.handle = h
        mu = (ctypes.c_double * 3)()
        _capi.check(self.lib.gs_masked_info(h, mu, None), "gs_masked_info")
        self.mu = np.array(mu[:])
        self.v = torch.zeros((self.F, self.Npix), dtype=torch.float64, device=device)
        self._acc = torch.zeros(1, dtype=torch.int32, device=device)
        self._lr = torch.zeros(1, dtype=torch.float64, device=device)

    def __del__(self):
        _capi.park(dict(self.__dict__))       # inside a capture: tensors freed after it
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            _capi.release(self.lib.gs_masked_destroy, h)
            self.handle = None

    # -- conversions -------------------------------------------------------------------
    def _dl(self, all_dls):
        specs = SPECS[self.F]
        arr = np.stack([np.asarray(all_dls[s], dtype=np.float64)[: self.L + 1] for s in specs])
        return torch.from_numpy(np.ascontiguousarray(arr)).to(self.device)

    def _s(self, s):
        if isinstance(s, torch.Tensor):
            return s.to(self.device, torch.float64).contiguous().clone()
        if isinstance(s, np.ndarray):
            return torch.from_numpy(np.ascontiguousarray(s, dtype=np.float64).reshape(self.F, self.NR)).to(self.device)
        return torch.from_numpy(np.ascontiguousarray(np.stack([np.asarray(s[k], dtype=np.float64)
                                                              for k in FIELDS[self.F]]))).to(self.device)

    def _out(self, s):
        a = s.cpu().numpy()
        return {k: a[i].copy() for i, k in enumerate(FIELDS[self.F])}

    def second_part_grad(self):
        out = torch.empty((self.F, self.NR), dtype=torch.float64, device=self.device)
        _capi.check(self.lib.gs_masked_info(self.handle, None, _capi.ptr(out)), "gs_masked_info")
        return out

    # -- replay draws (reference order) -----------------------------------
    def _pix(self, n):
        return np.stack([np.stack([np.random.normal(size=self.Npix) for _ in range(self.F)]) for _ in range(n)])

    def _slots(self):
        return np.stack([np.random.normal(size=self.NR) for _ in range(self.F)])

    def _replay(self, kind):
        zv = zs = zm = um = None
        if kind == _capi.GS_MCR_AUX or kind == _capi.GS_MCR_AUX_MALA:
            v, s = [], []
            for _ in range(self.n_gibbs):
                v.append(self._pix(1)[0])
                s.append(self._slots())
            zv, zs = np.stack(v), np.stack(s)
        elif kind == _capi.GS_MCR_OVERRELAX:
            v, s = [self._pix(1)[0]], []
            for _ in range(self.n_gibbs):
                s.append(self._slots())
                v.append(self._pix(1)[0])
                s.append(self._slots())
            zv, zs = np.stack(v), np.stack(s)
        if kind in (_capi.GS_MCR_MALA, _capi.GS_MCR_AUX_MALA):
            zm = self._slots()
            um = np.array([np.random.uniform()])
        dev = lambda a: None if a is None else torch.from_numpy(np.ascontiguousarray(a)).to(self.device)
        return dev(zv), dev(zs), dev(zm), dev(um)

    # -- the device step -------------------------------------------------------------------
    def step(self, kind, dl, s, iteration=None):
        """One CR call on device tensors (dl [nspec, L+1] unbinned, s [F, NR] in place)."""
        it = self.iteration if iteration is None else int(iteration)
        zv = zs = zm = um = None
        if self.rng == "replay":
            zv, zs, zm, um = self._replay(kind)
        _capi.check(self.lib.gs_masked_cr(self.handle, kind, _capi.ptr(dl), _capi.ptr(s), _capi.ptr(self.v),
                                          _capi.ptr(zv), _capi.ptr(zs), _capi.ptr(zm), _capi.ptr(um), self.seed, it,
                                          self.chain, _capi.ptr(self._acc), _capi.ptr(self._lr),
                                          _capi.stream_ptr()), "gs_masked_cr")
        return s

    def _run(self, kind, all_dls, s_old):
        s = self._s(s_old)
        self.step(kind, self._dl(all_dls), s)
        return self._out(s), int(self._acc.item())

    # -- reference surface ----------------------------------------------------------------
    def sample_gibbs_change_variable(self, all_dls, old_s):
        return self._run(_capi.GS_MCR_AUX, all_dls, old_s)

    def overrelaxation_sampler(self, all_dls, old_s):
        return self._run(_capi.GS_MCR_OVERRELAX, all_dls, old_s)

    def sample_mala(self, all_dls, s_old):
        return self._run(_capi.GS_MCR_MALA, all_dls, s_old)

    def compute_gradient_mala(self, all_dls, s_old):
        s = self._s(s_old)
        grad = torch.empty_like(s)
        pix = torch.empty((self.F, self.Npix), dtype=torch.float64, device=self.device)
        dl = self._dl(all_dls)
        _capi.check(self.lib.gs_masked_gradient(self.handle, _capi.ptr(dl), _capi.ptr(s),
                                                _capi.ptr(grad), _capi.ptr(pix), _capi.stream_ptr()),
                    "gs_masked_gradient")
        g, p = grad.cpu().numpy(), pix.cpu().numpy()
        return (*[g[i] for i in range(self.F)], *[p[i] for i in range(self.F)])

    # -- f1: PCG ------------------------------------------------------------------------
    def pcg_rhs(self, dl, iteration=None):
        """right-hand side b A^T N^-1 d + fluctuations (device tensor [F, NR])."""
        it = self.iteration if iteration is None else int(iteration)
        zv = zs = None
        if self.rng == "replay":
            if self.F == 1:           # TT (CenteredGibbs.py:153-155): z_alm, then z_pix
                zs = torch.from_numpy(np.ascontiguousarray(self._slots())).to(self.device)
                zv = torch.from_numpy(np.ascontiguousarray(self._pix(1)[0])).to(self.device)
            else:                     # CenteredGibbs.py:467-478: z_Q, z_U, then z_E, z_B
                zv = torch.from_numpy(np.ascontiguousarray(self._pix(1)[0])).to(self.device)
                zs = torch.from_numpy(np.ascontiguousarray(self._slots())).to(self.device)
        rhs = torch.empty((self.F, self.NR), dtype=torch.float64, device=self.device)
        _capi.check(self.lib.gs_masked_pcg_rhs(self.handle, _capi.ptr(dl), _capi.ptr(zv), _capi.ptr(zs), self.seed,
                                               it, self.chain, _capi.ptr(rhs), _capi.stream_ptr()),
                    "gs_masked_pcg_rhs")
        return rhs

    def pcg_solve(self, dl, rhs, x=None, tol=None, maxiter=None):
        guess = x is not None
        x = torch.empty_like(rhs) if x is None else x
        iters = ctypes.c_int()
        res = ctypes.c_double()
        _capi.check(self.lib.gs_masked_pcg_solve(self.handle, _capi.ptr(dl), _capi.ptr(rhs), _capi.ptr(x),
                                                 int(guess), self.pcg_accuracy if tol is None else float(tol),
                                                 self.pcg_maxiter if maxiter is None else int(maxiter),
                                                 ctypes.byref(iters), ctypes.byref(res), _capi.stream_ptr()),
                    "gs_masked_pcg_solve")
        self.pcg_iterations.append(iters.value)
        self.pcg_residual = res.value
        syncs = ctypes.c_int()
        _capi.check(self.lib.gs_masked_pcg_info(self.handle, ctypes.byref(syncs)), "gs_masked_pcg_info")
        self.pcg_syncs.append(syncs.value)          # host synchronisations of this solve (one per batch)
        return x

    def pcg_apply(self, dl, x, out=None):
        """out = Q x, the PCG system operator (qcinv fwd_op, CenteredGibbs.py:631,655)."""
        out = torch.empty_like(x) if out is None else out
        _capi.check(self.lib.gs_masked_pcg_apply(self.handle, _capi.ptr(dl), _capi.ptr(x), _capi.ptr(out),
                                                 _capi.stream_ptr()), "gs_masked_pcg_apply")
        return out

    def rj_step(self, dl, s, iteration=None):
        """RJPO CR on device tensors (sample_mask_rj, CenteredGibbs.py:606-674), s
        [F, NR] updated in place: the PCG right-hand side with fresh fluctuations
        (the draws of sample_mask, :622-643), the solve started from -s (:645-650),
        then log_proba = -sum (rhs - Q x) . (s - x) and log u < log_proba on the
        device (:652-672).  Replay: the uniform is np.random.uniform() after the
        normals, the reference's order."""
        it = self.iteration if iteration is None else int(iteration)
        rhs = self.pcg_rhs(dl, iteration=it)
        um = None
        if self.rng == "replay":
            um = torch.tensor([np.random.uniform()], dtype=torch.float64, device=self.device)
        x = self.pcg_solve(dl, rhs, x=-s)
        _capi.check(self.lib.gs_masked_rj_accept(self.handle, _capi.ptr(dl), _capi.ptr(rhs), _capi.ptr(x),
                                                 _capi.ptr(s), _capi.ptr(um), self.seed, it, self.chain,
                                                 _capi.ptr(self._acc), _capi.ptr(self._lr), _capi.stream_ptr()),
                    "gs_masked_rj_accept")
        return s

    def sample_mask_rj(self, all_dls, s_old):
        """CenteredGibbs.py:606-674: (map, 1) when the RJPO proposal is accepted,
        (s_old, 0) otherwise."""
        s = self._s(s_old)
        self.rj_step(self._dl(all_dls), s)
        return self._out(s), int(self._acc.item())

    def tt_fullsky(self, dl, noncentered=False, iteration=None, out=None):
        """temperature full-sky CR from the pixel map (gs_masked_tt_fullsky):
        CenteredGibbs.py:108-132 or NonCenteredGibbs.py:22-38; replay draws
        z_alm then z_pix."""
        it = self.iteration if iteration is None else int(iteration)
        zv = zs = None
        if self.rng == "replay":
            zs = torch.from_numpy(np.ascontiguousarray(self._slots())).to(self.device)
            zv = torch.from_numpy(np.ascontiguousarray(self._pix(1)[0])).to(self.device)
        out = torch.empty((1, self.NR), dtype=torch.float64, device=self.device) if out is None else out
        _capi.check(self.lib.gs_masked_tt_fullsky(self.handle, int(bool(noncentered)), _capi.ptr(dl), _capi.ptr(zv),
                                                  _capi.ptr(zs), self.seed, it, self.chain, _capi.ptr(out),
                                                  _capi.stream_ptr()), "gs_masked_tt_fullsky")
        return out

    def sample_mask(self, all_dls):
        """CenteredGibbs.py:448-491: PCG constrained realisation; accept 1."""
        dl = self._dl(all_dls)
        x = self.pcg_solve(dl, self.pcg_rhs(dl))
        return self._out(x), 1

    def last_log_ratio(self):
        return float(self._lr.item())

    def sample(self, all_dls, s_old=None):
        """CenteredGibbs.py:828-850 (masked): the flag ladder."""
        if s_old is None:
            return self.sample_mask(all_dls)
        if self.gibbs_cr and self.overrelaxation:
            return self.overrelaxation_sampler(all_dls, s_old)
        if self.gibbs_cr and not self.ula:
            return self.sample_gibbs_change_variable(all_dls, s_old)
        if self.gibbs_cr and self.ula:
            return self._run(_capi.GS_MCR_AUX_MALA, all_dls, s_old)
        if self.rj:
            return self.sample_mask_rj(all_dls, s_old)
        if self.ula:
            return self.sample_mala(all_dls, s_old)
        return self.sample_mask(all_dls)


KIND_PCG = -1     # sample_mask (f1), driven from the host (CG loop)
KIND_RJ = -2      # sample_mask_rj (RJPO: the PCG from -s_old + an accept step)


def cr_kind(gibbs_cr, overrelaxation, ula, rj=False):
    """The flag ladder of CenteredGibbs.py:828-850 for a masked run with a map
    (rj: the RJPO branch of :837-838, which HEAD disables)."""
    if gibbs_cr and overrelaxation:
        return _capi.GS_MCR_OVERRELAX
    if gibbs_cr and not ula:
        return _capi.GS_MCR_AUX
    if gibbs_cr and ula:
        return _capi.GS_MCR_AUX_MALA
    if rj:
        return KIND_RJ
    if ula:
        return _capi.GS_MCR_MALA
    return KIND_PCG


class MaskedRunner:
    """GibbsSampler.run_polarization (GibbsSampler.py:118-180) for a masked run on
    one chain: per iteration the masked CR (MaskedCR, the a12 ladder) and the
    centered C_l draw (gs_sweep_stats + gs_cls_draw), everything resident on
    the device.  The reference's first CR (GibbsSampler.py:136-138) is the
    qcinv PCG (row f1); the start map is given instead (``s_init``)."""

    def __init__(self, cr, bins, kind=None):
        from .engine import GibbsPlan
        self.cr = cr
        self.kind = cr_kind(cr.gibbs_cr, cr.overrelaxation, cr.ula, cr.rj) if kind is None else kind
        F = cr.F
        self.spectra = ("EE", "BB") if F == 2 else ("TT", "EE", "BB", "TE")
        self.bins = {s: np.asarray(bins[s]) for s in self.spectra}
        self.plan = GibbsPlan(cr.L, cr.nside, F, 1, cr.bl, [1.0] * F, self.bins, chain0=cr.chain)
        self.d0 = self.plan.zeros(F, cr.NR)
        L = cr.L
        idx = np.full((len(self.spectra), L + 1), -1, dtype=np.int64)
        for k, sp in enumerate(self.spectra):
            b = self.bins[sp]
            for i in range(len(b) - 1):
                idx[k, b[i]:min(b[i + 1], L + 1)] = i
        self._idx = torch.from_numpy(np.maximum(idx, 0)).to(cr.device)
        self._valid = torch.from_numpy(idx >= 0).to(cr.device)

    def _unfold(self, binned_t):
        """utils.unfold_bins on the device: binned [1, nspec, maxbins] -> [nspec, L+1]."""
        return torch.where(self._valid, torch.gather(binned_t[0], 1, self._idx), 0.0).contiguous()

    def run(self, dls_init, n_iter, s_init):
        """The loop stays on the device: D_l, the accept flags and the histories are
        device tensors until the end (one host transfer per run instead of a sync
        and two copies per iteration); the per-iteration CR / C_l times come from
        events read after the loop."""
        cr, plan = self.cr, self.plan
        binned0 = {s: np.asarray(dls_init[s], dtype=np.float64) for s in self.spectra}
        binned = plan.dl_tensor(binned0)
        hist, acc, evs = [binned], [], []
        if s_init is None:
            # GibbsSampler.py:136-138: the first CR is sample(dls) without a map ->
            # the PCG (sample_mask), iteration 0 of the native streams
            dl0 = self._unfold(binned)
            s = cr.pcg_solve(dl0, cr.pcg_rhs(dl0, iteration=0))
        else:
            s = cr._s(s_init)
        one = torch.ones(1, dtype=torch.int32, device=cr.device)
        for i in range(n_iter):
            it = i + 1
            cr.iteration = it
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            ev[0].record()
            dl = self._unfold(binned)
            if self.kind == KIND_PCG:
                s = cr.pcg_solve(dl, cr.pcg_rhs(dl, iteration=it))
                acc.append(one)
            elif self.kind == KIND_RJ:
                cr.rj_step(dl, s, iteration=it)
                acc.append(cr._acc.reshape(1).clone())
            else:
                cr.step(self.kind, dl, s, iteration=it)
                acc.append(cr._acc.reshape(1).clone())
            ev[1].record()
            stats = plan.sweep_stats(self.d0, s[None])
            var = plan.replay_invgamma() if cr.rng == "replay" else None
            binned = plan.cls_draw(stats, var, seed=cr.seed, iteration=it)
            ev[2].record()
            hist.append(binned)
            evs.append(ev)
        self.s = s
        torch.cuda.synchronize()
        t_cr = np.array([e[0].elapsed_time(e[1]) * 1e-3 for e in evs])
        t_cls = np.array([e[1].elapsed_time(e[2]) * 1e-3 for e in evs])
        H = torch.cat(hist).cpu().numpy()                     # [n_iter + 1, nspec, maxbins]
        A = torch.cat(acc).cpu().numpy().astype(np.int64) if acc else np.zeros(0, dtype=np.int64)
        h = {sp: H[:, k, :len(self.bins[sp]) - 1].copy() for k, sp in enumerate(self.spectra)}
        return h, A, t_cr, t_cls


# ---------------------------------------------------------------------------------------
# f2: pixel-domain non-centred likelihood (masked NonCenteredGibbs / ASIS)
# ---------------------------------------------------------------------------------------
class PixelMH:
    """PolarizationNonCenteredClsSampler.sample with all_sph=False
    (NonCenteredGibbs.py:401-445; TT: NonCenteredClsSampler.sample): truncated-
    normal proposals for every bin (gs_mh_propose), then the Metropolis blocks
    scored with the whole-map likelihood -1/2 sum_pix N^-1 (d - A b C^1/2 s_nc)^2
    (compute_log_likelihood, NonCenteredGibbs.py:333-355) and decided in the
    reference's order ON THE DEVICE by gs_masked_pixel_mh: the likelihood
    change of every block comes from one shared-recurrence block synthesis and
    one weighted Gram pass instead of one SHT and one host round trip per
    block.  The accept flags are read back once per sweep.
    Replay: numpy draws truncnorm EE, BB then one uniform per block attempt,
    the reference's order (the likelihood draws nothing)."""

    def __init__(self, cr, bins, blocks, proposal_variances, n_iter_metropolis=1):
        from .engine import GibbsPlan, MH_ORDER
        if cr.F == 3:
            raise NotImplementedError("the pixel-domain NC sampler is the reference's EB / TT model "
                                      "(PolarizationNonCenteredClsSampler, NonCenteredClsSampler); TEB is not "
                                      "defined there")
        F = cr.F
        self.cr = cr
        self.spectra = SPECS[F]
        self.order = MH_ORDER[F]
        self.bins = {s: np.asarray(bins[s]) for s in self.spectra}
        self.blocks = {s: np.asarray(blocks[s]) for s in self.spectra}
        self.n_iter = int(n_iter_metropolis)
        self.plan = GibbsPlan(cr.L, cr.nside, F, 1, cr.bl, [1.0] * F, self.bins, blocks=self.blocks,
                              proposal_variances=proposal_variances, chain0=cr.chain,
                              n_iter_metropolis=self.n_iter)
        L = cr.L
        idx = np.full((F, L + 1), -1, dtype=np.int64)
        for k, s in enumerate(self.spectra):
            b = self.bins[s]
            for i in range(len(b) - 1):
                idx[k, b[i]:min(b[i + 1], L + 1)] = i
        self._idx = torch.from_numpy(np.maximum(idx, 0)).to(cr.device)
        self._valid = torch.from_numpy(idx >= 0).to(cr.device)
        self._lik = torch.zeros(1, dtype=torch.float64, device=cr.device)
        # block tables of gs_masked_pixel_mh, in decision order (spectra in MH order)
        blk = np.full((F, L + 1), -1, dtype=np.int32)
        lmax_, field, brange, self._acc_layout = [], [], [], []
        for s in self.order:
            k = self.spectra.index(s)
            edges, nb = self.blocks[s], len(self.bins[s]) - 1
            for bi in range(len(edges) - 1):
                lo, hi = int(edges[bi]), min(int(edges[bi + 1]), nb)
                l0, l1 = (int(self.bins[s][lo]), int(self.bins[s][hi])) if hi > lo else (0, 0)
                kg = len(field)
                blk[k, l0:min(l1, L + 1)] = kg
                lmax_.append(min(l1, L + 1) - 1 if l1 > l0 else -1)
                field.append(k)
                brange += [lo, max(hi, lo)]
            self._acc_layout.append((s, (len(edges) - 1) * self.n_iter))
        self.K = len(field)
        dev = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).to(cr.device)
        self._blk, self._blk_lmax, self._blk_field, self._blk_bins = dev(blk), dev(lmax_), dev(field), dev(brange)
        self._acc = torch.zeros(max(self.K * self.n_iter, 1), dtype=torch.int32, device=cr.device)

    def unfold(self, binned_t):
        """utils.unfold_bins on the device: [nspec, maxbins] -> [nspec, L+1]."""
        return torch.where(self._valid, torch.gather(binned_t, 1, self._idx), 0.0).contiguous()

    def noncentre(self, dl_unbinned, s):
        """s_nc = C^-1/2 s (zero where C = 0; NonCenteredGibbs.py:186-191, ASIS.py:184-190)."""
        out = torch.empty_like(s)
        _capi.check(self.cr.lib.gs_masked_center(self.cr.handle, _capi.ptr(dl_unbinned), -1, _capi.ptr(s),
                                                 _capi.ptr(out), _capi.stream_ptr()), "gs_masked_center")
        return out

    def centre(self, dl_unbinned, s):
        """C^1/2 s."""
        out = torch.empty_like(s)
        _capi.check(self.cr.lib.gs_masked_center(self.cr.handle, _capi.ptr(dl_unbinned), 1, _capi.ptr(s),
                                                 _capi.ptr(out), _capi.stream_ptr()), "gs_masked_center")
        return out

    def loglik_t(self, dl_unbinned, s_nc):
        _capi.check(self.cr.lib.gs_masked_nc_loglik(self.cr.handle, _capi.ptr(dl_unbinned), _capi.ptr(s_nc),
                                                    _capi.ptr(self._lik), _capi.stream_ptr()),
                    "gs_masked_nc_loglik")
        return self._lik

    def compute_log_likelihood(self, dls, s_nonCentered):
        """NonCenteredGibbs.py:333-355 (binned dict, dict / array map) -> float."""
        bt = self.plan.dl_tensor(dls)[0]
        return float(self.loglik_t(self.unfold(bt), self.cr._s(s_nonCentered)).item())

    def sweep_t(self, s_nc, binned_t, iteration):
        """one sweep on device tensors, no host synchronisation: binned_t
        [nspec, maxbins] -> (updated copy, accept flags [K * n_iter] int32 in
        decision order; the flags tensor is reused by the next sweep)."""
        plan, cr = self.plan, self.cr
        dl = binned_t[None].contiguous()
        if cr.rng == "replay":
            up, ua = plan.replay_mh_uniforms()
            prop, logr, _ = plan.mh_propose(dl, up, seed=cr.seed, iteration=iteration)
        else:
            prop, logr, ua = plan.mh_propose(dl, None, seed=cr.seed, iteration=iteration, with_uniforms=True)
        prop0, logr0 = prop[0].contiguous(), logr[0].contiguous()
        cur = binned_t.clone()
        # every temporary stays referenced until the launch is enqueued (a freed
        # tensor's block is handed to the next allocation)
        dl_cur, dl_prop, u0 = self.unfold(cur), self.unfold(prop0), ua[0].contiguous()
        _capi.check(self.cr.lib.gs_masked_pixel_mh(
            cr.handle, self.K, self.n_iter, plan.maxbins, _capi.ptr(self._blk), _capi.ptr(self._blk_lmax),
            _capi.ptr(self._blk_field), _capi.ptr(self._blk_bins), _capi.ptr(s_nc), _capi.ptr(dl_cur),
            _capi.ptr(dl_prop), _capi.ptr(logr0), _capi.ptr(u0), _capi.ptr(prop0),
            _capi.ptr(cur), _capi.ptr(self._acc), _capi.stream_ptr()), "gs_masked_pixel_mh")
        return cur, self._acc

    def split_accept(self, flags):
        a = flags.cpu().numpy()
        out, off = {}, 0
        for s, n in self._acc_layout:
            out[s] = [int(v) for v in a[off:off + n]]
            off += n
        return out

    def sample_t(self, s_nc, binned_t, iteration):
        """one sweep on device tensors: binned_t [nspec, maxbins] (updated copy
        returned), s_nc [nspec, NR]; returns (binned_t, accept dict of lists)."""
        cur, flags = self.sweep_t(s_nc, binned_t, iteration)
        return cur, self.split_accept(flags)

    def sample(self, s_nonCentered, binned_dls_old, iteration=None):
        """reference surface: dict maps / binned dicts in, (binned dict, accept dict) out."""
        it = self.cr.iteration if iteration is None else int(iteration)
        bt = self.plan.dl_tensor(binned_dls_old)[0]
        cur, acc = self.sample_t(self.cr._s(s_nonCentered), bt, it)
        return self.plan.dl_dicts(cur[None])[0], acc


class MaskedMHRunner:
    """Masked non-centred and interweaving drivers on one chain:

    kind "noncentered": NonCenteredClsSampler.run_polarization
      (NonCenteredGibbs.py:529-571) -- per iteration the PCG CR in the centred
      parametrisation, s_nc = C^-1/2 s (sample_mask, :178-196), pixel MH.
    kind "asis": ASIS.run_polarization (ASIS.py:134-226) -- the masked CR
      ladder (PCG, or the a9-a12 samplers with a start map from the PCG),
      centred C_l draw, non-centring with the intermediate D_l, pixel MH, and
      the re-centring of ASIS.py:201-203 (``quirk``: the reference scales the
      CENTRED map by C_new^1/2; otherwise C_new^1/2 s_nc)."""

    def __init__(self, kind, cr, bins, blocks, proposal_variances, n_iter_metropolis=1, cr_kind_=KIND_PCG,
                 quirk=True):
        if kind not in ("noncentered", "asis"):
            raise ValueError(kind)
        self.kind, self.cr, self.quirk = kind, cr, bool(quirk)
        self.mh = PixelMH(cr, bins, blocks, proposal_variances, n_iter_metropolis)
        self.cr_kind = cr_kind_ if kind == "asis" else KIND_PCG
        self.plan = self.mh.plan
        self.d0 = self.plan.zeros(cr.F, cr.NR)

    def _pcg(self, dl, it):
        return self.cr.pcg_solve(dl, self.cr.pcg_rhs(dl, iteration=it))

    def run(self, dls_init, n_iter, s_init=None):
        """n_iter iterations from dls_init (binned dict).  s_init: continue from
        this map instead of the reference's PCG start map (ASIS.py:153-156).
        The loop stays on the device (D_l, accept flags and histories are device
        tensors until the end; the stage times come from events read after it)."""
        cr, mh, plan = self.cr, self.mh, self.plan
        cur = plan.dl_tensor({s: np.asarray(dls_init[s], dtype=np.float64) for s in mh.spectra})[0]
        hist, flags, acc_cr, evs = [cur], [], [], []
        dl = mh.unfold(cur)
        s = None
        if s_init is not None:
            s = cr._s(s_init)
        elif self.kind == "asis" and self.cr_kind != KIND_PCG:
            s = self._pcg(dl, 0)          # ASIS.py:153-156: the start map from the PCG
        for i in range(n_iter):
            it = i + 1
            cr.iteration = it
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            ev[0].record()
            if self.kind == "noncentered":
                s = self._pcg(dl, it)
                s_nc = mh.noncentre(dl, s)
                ev[1].record()
                ev[2].record()
                cur, f = mh.sweep_t(s_nc, cur, it)
                dl = mh.unfold(cur)
            else:
                if self.cr_kind == KIND_PCG:
                    s = self._pcg(dl, it)
                else:
                    cr.step(self.cr_kind, dl, s, iteration=it)
                    acc_cr.append(cr._acc.reshape(1).clone())
                ev[1].record()
                stats = plan.sweep_stats(self.d0[None], s[None])
                var = plan.replay_invgamma() if cr.rng == "replay" else None
                tmp = plan.cls_draw(stats, var, seed=cr.seed, iteration=it)[0]
                dl_tmp = mh.unfold(tmp)
                s_nc = mh.noncentre(dl_tmp, s)
                ev[2].record()
                cur, f = mh.sweep_t(s_nc, tmp, it)
                dl = mh.unfold(cur)
                s = mh.centre(dl, s if self.quirk else s_nc)
            ev[3].record()
            flags.append(f.clone())           # sweep_t reuses its flags tensor
            hist.append(cur)
            evs.append(ev)
        self.s = s
        torch.cuda.synchronize()
        el = lambda e, a, b: e[a].elapsed_time(e[b]) * 1e-3
        t_it = np.array([el(e, 0, 3) for e in evs])
        t_cr = np.array([el(e, 0, 1) for e in evs])
        t_cls = np.array([el(e, 1, 2) for e in evs])
        t_nc = np.array([el(e, 2, 3) for e in evs])
        H = torch.stack(hist).cpu().numpy()                   # [n_iter + 1, nspec, maxbins]
        h = {sp: H[:, k, :len(mh.bins[sp]) - 1].copy() for k, sp in enumerate(mh.spectra)}
        acc = {sp: [] for sp in mh.spectra}
        if flags:
            Fl = torch.stack(flags).cpu().numpy()
            for row in Fl:
                off = 0
                for sp, n in mh._acc_layout:
                    acc[sp].append([int(v) for v in row[off:off + n]])
                    off += n
        a_cr = torch.cat(acc_cr).cpu().numpy().astype(np.int64) if acc_cr else None
        out = ({sp: np.array(v) for sp, v in h.items()}, {sp: np.array(v) for sp, v in acc.items()})
        return out + (a_cr, t_it, t_cr, t_cls, t_nc)
