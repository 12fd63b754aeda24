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

Chains: ``nchains`` = B > 1 runs B independent chains of the same data set in
one context (global ids chain .. chain + B - 1) -- the reference's SLURM array
of chains (job-script.sh:6-8) as one batch whose transforms are batched SHTs
(one launch per stage for all B maps).  Device arrays then carry a leading
chain axis ([B, F, NR], [B, nspec, L+1], ...); with B = 1 the shapes are the
one-chain ones.  Chain b of a batch is bit-identical to a one-chain context of
chain id chain + b that runs the same Legendre stage: ``sht_mode="auto"``
resolves to the matrix-core tables for B >= 4 on small maps and to the
recurrence otherwise (the two agree to ~1e-12 relative, not bit for bit), so
pass "recurrence" or "mfma" explicitly when a batch must reproduce a one-chain
run; ``sht_tables`` reports the resolved path.  Replay draws for B > 1 are
chain-major: each chain's reference-order draws in turn.
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
                 device="cuda", pcg_accuracy=1.0e-5, pcg_maxiter=4000, rj=False, nchains=1, sht_mode="auto"):
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
        self.B = int(nchains)
        if self.B < 1:
            raise ValueError("nchains >= 1")
        self.pcg_iterations = []          # per solve: the CG iterations (mean over the batch's chains)
        self.pcg_iterations_chains = []   # per solve: every chain's count
        self.pcg_launched = []            # per solve: CG iterations launched (the slowest chain's)
        self.pcg_work = []                # per solve: chain-iterations transformed (converged chains dropped)
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
        desc.nchains = self.B
        # the Legendre stage: "auto" (matrix-core tables for >= 4 chains on small
        # maps), "recurrence" (on-the-fly VALU kernels) or "mfma"
        desc.sht_mode = {"auto": 0, "recurrence": 1, "mfma": 2}[sht_mode]
        h = ctypes.c_void_p()
        _capi.check(self.lib.gs_masked_create(ctypes.byref(desc), _capi.ptr(self._maps), _capi.ptr(self._inv),
                                              ctypes.byref(h)), "gs_masked_create")
        self.handle = h
        mu = (ctypes.c_double * 3)()
        _capi.check(self.lib.gs_masked_info(h, mu, None), "gs_masked_info")
        self.mu = np.array(mu[:])
        self.v = torch.zeros(self._shape(self.F, self.Npix), dtype=torch.float64, device=device)
        self._acc = torch.zeros(self.B, dtype=torch.int32, device=device)
        self._lr = torch.zeros(self.B, dtype=torch.float64, device=device)

    @property
    def sht_tables(self):
        """True when the context's transforms run the matrix-core table path."""
        return bool(self.lib.gs_masked_sht_tables(self.handle))

    @property
    def ring_classes(self):
        """(pairs without weight, pairs with varying ring weights, pairs with one
        weight per ring) of the context's N^-1 (gs_masked_ring_classes)."""
        c = (ctypes.c_int * 3)()
        _capi.check(self.lib.gs_masked_ring_classes(self.handle, c), "gs_masked_ring_classes")
        return tuple(int(v) for v in c)

    def __del__(self):
        if getattr(_capi, "park", None) is None:    # interpreter teardown: the driver frees everything
            return
        _capi.park(dict(self.__dict__))       # inside a capture: tensors freed after it
        h = getattr(self, "handle", None)
        if h is not None and h.value:
            _capi.release(self.lib.gs_masked_destroy, h)
            self.handle = None

    # -- conversions -------------------------------------------------------------------
    def _shape(self, *tail):
        """a per-chain array's shape: the one-chain shape, or [B, ...] for a batch"""
        return tail if self.B == 1 else (self.B,) + tail

    def _dl(self, all_dls):
        """D_l dict (every chain) or list of B dicts -> device [B?, nspec, L+1]."""
        specs = SPECS[self.F]
        one = lambda d: np.stack([np.asarray(d[s], dtype=np.float64)[: self.L + 1] for s in specs])
        if isinstance(all_dls, (list, tuple)):
            arr = np.stack([one(d) for d in all_dls])
        else:
            arr = one(all_dls)
            if self.B > 1:
                arr = np.broadcast_to(arr, (self.B,) + arr.shape)
        return torch.from_numpy(np.ascontiguousarray(arr)).to(self.device).reshape(self._shape(len(specs), self.L + 1))

    def _s(self, s):
        if isinstance(s, torch.Tensor):
            return s.to(self.device, torch.float64).contiguous().clone().reshape(self._shape(self.F, self.NR))
        if isinstance(s, np.ndarray):
            return torch.from_numpy(np.ascontiguousarray(s, dtype=np.float64).reshape(
                self._shape(self.F, self.NR))).to(self.device)
        one = lambda d: np.stack([np.asarray(d[k], dtype=np.float64) for k in FIELDS[self.F]])
        arr = np.stack([one(d) for d in s]) if isinstance(s, (list, tuple)) else one(s)
        return torch.from_numpy(np.ascontiguousarray(arr).reshape(self._shape(self.F, self.NR))).to(self.device)

    def _out(self, s):
        a = s.cpu().numpy().reshape(self.B, self.F, self.NR)
        out = [{k: a[b, i].copy() for i, k in enumerate(FIELDS[self.F])} for b in range(self.B)]
        return out[0] if self.B == 1 else out

    def _flags(self, t):
        a = t.cpu().numpy()
        return int(a[0]) if self.B == 1 else a.astype(np.int64)

    def second_part_grad(self):
        out = torch.empty((self.F, self.NR), dtype=torch.float64, device=self.device)
        _capi.check(self.lib.gs_masked_info(self.handle, None, _capi.ptr(out)), "gs_masked_info")
        return out

    # -- replay draws (reference order; chain-major for a batch) --------
    def _pix(self, n):
        return np.stack([np.stack([np.random.normal(size=self.Npix) for _ in range(self.F)]) for _ in range(n)])

    def _slots(self):
        return np.stack([np.random.normal(size=self.NR) for _ in range(self.F)])

    def _replay_one(self, kind):
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
        return zv, zs, zm, um

    def _dev(self, a):
        return None if a is None else torch.from_numpy(np.ascontiguousarray(a)).to(self.device)

    def _replay(self, kind):
        per = [self._replay_one(kind) for _ in range(self.B)]
        return tuple(self._dev(None if per[0][k] is None else np.stack([p[k] for p in per])) for k in range(4))

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
        return self._out(s), self._flags(self._acc)

    # -- reference surface ----------------------------------------------------------------
    def sample_gibbs_change_variable(self, all_dls, old_s):
        return self._run(_capi.GS_MCR_AUX, all_dls, old_s)

    def overrelaxation_sampler(self, all_dls, old_s):
        return self._run(_capi.GS_MCR_OVERRELAX, all_dls, old_s)

    def sample_mala(self, all_dls, s_old):
        return self._run(_capi.GS_MCR_MALA, all_dls, s_old)

    def compute_gradient_mala(self, all_dls, s_old):
        if self.B != 1:
            raise NotImplementedError("compute_gradient_mala: the reference surface's one-chain form")
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
    def _rhs_draws_one(self):
        """one chain's PCG fluctuation normals in the reference's order -> (z_pix, z_slot)"""
        if self.F == 1:                   # TT (CenteredGibbs.py:153-155): z_alm, then z_pix
            zs = self._slots()
            return self._pix(1)[0], zs
        zv = self._pix(1)[0]              # CenteredGibbs.py:467-478: z_Q, z_U, then z_E, z_B
        return zv, self._slots()

    def pcg_rhs(self, dl, iteration=None, draws=None):
        """right-hand side b A^T N^-1 d + fluctuations (device tensor [F, NR]).
        draws: replay normals already drawn, a list of B (z_pix, z_slot) pairs."""
        it = self.iteration if iteration is None else int(iteration)
        zv = zs = None
        if self.rng == "replay":
            per = draws if draws is not None else [self._rhs_draws_one() for _ in range(self.B)]
            zv, zs = self._dev(np.stack([p[0] for p in per])), self._dev(np.stack([p[1] for p in per]))
        rhs = torch.empty(self._shape(self.F, self.NR), dtype=torch.float64, device=self.device)
        _capi.check(self.lib.gs_masked_pcg_rhs(self.handle, _capi.ptr(dl), _capi.ptr(zv), _capi.ptr(zs), self.seed,
                                               it, self.chain, _capi.ptr(rhs), _capi.stream_ptr()),
                    "gs_masked_pcg_rhs")
        return rhs

    def pcg_solve(self, dl, rhs, x=None, tol=None, maxiter=None):
        guess = x is not None
        x = torch.empty_like(rhs) if x is None else x
        iters = (ctypes.c_int * self.B)()
        res = (ctypes.c_double * self.B)()
        _capi.check(self.lib.gs_masked_pcg_solve(self.handle, _capi.ptr(dl), _capi.ptr(rhs), _capi.ptr(x),
                                                 int(guess), self.pcg_accuracy if tol is None else float(tol),
                                                 self.pcg_maxiter if maxiter is None else int(maxiter),
                                                 iters, res, _capi.stream_ptr()),
                    "gs_masked_pcg_solve")
        its = [int(v) for v in iters]
        self.pcg_iterations.append(its[0] if self.B == 1 else float(np.mean(its)))
        self.pcg_iterations_chains.append(its)
        self.pcg_residual = res[0] if self.B == 1 else [float(v) for v in res]
        syncs, launched = ctypes.c_int(), ctypes.c_int()
        _capi.check(self.lib.gs_masked_pcg_info2(self.handle, ctypes.byref(syncs), ctypes.byref(launched)),
                    "gs_masked_pcg_info2")
        self.pcg_syncs.append(syncs.value)          # host synchronisations of this solve (one per batch)
        self.pcg_launched.append(launched.value)    # iterations launched (the batch's slowest chain)
        work = ctypes.c_longlong()
        _capi.check(self.lib.gs_masked_pcg_work(self.handle, ctypes.byref(work)), "gs_masked_pcg_work")
        self.pcg_work.append(work.value)
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
        normals, the reference's order; a batch draws chain b's normals and then
        its uniform before chain b + 1's (chain-major like every replay draw)."""
        it = self.iteration if iteration is None else int(iteration)
        um = per = None
        if self.rng == "replay":
            per, us = [], []
            for _ in range(self.B):
                per.append(self._rhs_draws_one())
                us.append(np.random.uniform())
            um = torch.tensor(us, dtype=torch.float64, device=self.device)
        rhs = self.pcg_rhs(dl, iteration=it, draws=per)
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
        return self._out(s), self._flags(self._acc)

    def tt_fullsky(self, dl, noncentered=False, iteration=None, out=None):
        """temperature full-sky CR from the pixel map (gs_masked_tt_fullsky):
        CenteredGibbs.py:108-132 or NonCenteredGibbs.py:22-38; replay draws
        z_alm then z_pix."""
        it = self.iteration if iteration is None else int(iteration)
        zv = zs = None
        if self.rng == "replay":
            zsl, zvl = [], []
            for _ in range(self.B):
                zsl.append(self._slots())
                zvl.append(self._pix(1)[0])
            zs, zv = self._dev(np.stack(zsl)), self._dev(np.stack(zvl))
        out = torch.empty(self._shape(1, self.NR), dtype=torch.float64, device=self.device) if out is None else out
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
        a = self._lr.cpu().numpy()
        return float(a[0]) if self.B == 1 else a

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


def _unfold_index(spectra, bins, L, device):
    """the (index, valid) pair of utils.unfold_bins on the device: row k, l -> bin"""
    idx = np.full((len(spectra), L + 1), -1, dtype=np.int64)
    for k, sp in enumerate(spectra):
        b = bins[sp]
        for i in range(len(b) - 1):
            idx[k, b[i]:min(b[i + 1], L + 1)] = i
    return torch.from_numpy(np.maximum(idx, 0)).to(device), torch.from_numpy(idx >= 0).to(device)


def _unfold_batch(binned_t, idx, valid):
    """utils.unfold_bins on the device: binned [B, nspec, maxbins] -> [B, nspec, L+1]."""
    B = binned_t.shape[0]
    g = torch.gather(binned_t, 2, idx.unsqueeze(0).expand(B, -1, -1))
    return torch.where(valid.unsqueeze(0), g, 0.0).contiguous()


class MaskedRunner:
    """GibbsSampler.run_polarization (GibbsSampler.py:118-180) for a masked run:
    per iteration the masked CR (MaskedCR, the a12 ladder) and the centered C_l
    draw (gs_sweep_stats + gs_cls_draw), everything resident on the device, for
    the context's B chains at once.  The reference's first CR
    (GibbsSampler.py:136-138) is the qcinv PCG (row f1); a start map may be
    given instead (``s_init``).  Histories: dict of [n_iter + 1, nbins] (B = 1)
    or [n_iter + 1, B, nbins]; accept flags [n_iter] or [n_iter, B]."""

    def __init__(self, cr, bins, kind=None):
        from .engine import GibbsPlan
        self.cr = cr
        self.kind = cr_kind(cr.gibbs_cr, cr.overrelaxation, cr.ula, cr.rj) if kind is None else kind
        F = cr.F
        self.spectra = ("EE", "BB") if F == 2 else ("TT", "EE", "BB", "TE")
        self.bins = {s: np.asarray(bins[s]) for s in self.spectra}
        self.plan = GibbsPlan(cr.L, cr.nside, F, cr.B, cr.bl, [1.0] * F, self.bins, chain0=cr.chain)
        self.d0 = self.plan.zeros(F, cr.NR)
        self._idx, self._valid = _unfold_index(self.spectra, self.bins, cr.L, cr.device)

    def _unfold(self, binned_t):
        """utils.unfold_bins on the device: binned [B, nspec, maxbins] -> [B?, nspec, L+1]."""
        return _unfold_batch(binned_t, self._idx, self._valid).reshape(self.cr._shape(len(self.spectra),
                                                                                       self.cr.L + 1))

    def run(self, dls_init, n_iter, s_init):
        """The loop stays on the device: D_l, the accept flags and the histories are
        device tensors until the end (one host transfer per run instead of a sync
        and two copies per iteration); the per-iteration CR / C_l times come from
        events read after the loop."""
        cr, plan = self.cr, self.plan
        if isinstance(dls_init, (list, tuple)):
            binned0 = [{s: np.asarray(d[s], dtype=np.float64) for s in self.spectra} for d in dls_init]
        else:
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
        ones = torch.ones(cr.B, dtype=torch.int32, device=cr.device)
        for i in range(n_iter):
            it = i + 1
            cr.iteration = it
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            ev[0].record()
            dl = self._unfold(binned)
            if self.kind == KIND_PCG:
                s = cr.pcg_solve(dl, cr.pcg_rhs(dl, iteration=it))
                acc.append(ones)
            elif self.kind == KIND_RJ:
                cr.rj_step(dl, s, iteration=it)
                acc.append(cr._acc.clone())
            else:
                cr.step(self.kind, dl, s, iteration=it)
                acc.append(cr._acc.clone())
            ev[1].record()
            stats = plan.sweep_stats(self.d0, s.reshape(cr.B, cr.F, cr.NR))
            var = plan.replay_invgamma() if cr.rng == "replay" else None
            binned = plan.cls_draw(stats, var, seed=cr.seed, iteration=it)
            ev[2].record()
            hist.append(binned)
            evs.append(ev)
        self.s = s
        torch.cuda.synchronize()
        t_cr = np.array([e[0].elapsed_time(e[1]) * 1e-3 for e in evs])
        t_cls = np.array([e[1].elapsed_time(e[2]) * 1e-3 for e in evs])
        H = torch.stack(hist).cpu().numpy()                   # [n_iter + 1, B, nspec, maxbins]
        A = torch.stack(acc).cpu().numpy().astype(np.int64) if acc else np.zeros((0, cr.B), dtype=np.int64)
        one = cr.B == 1
        h = {sp: (H[:, 0, k, :len(self.bins[sp]) - 1] if one else H[:, :, k, :len(self.bins[sp]) - 1]).copy()
             for k, sp in enumerate(self.spectra)}
        return h, (A[:, 0] if one else A), t_cr, t_cls


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
    the reference's order (the likelihood draws nothing).  A batched context
    (B chains) sweeps every chain (device tensors with a leading chain axis)."""

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
        self.plan = GibbsPlan(cr.L, cr.nside, F, cr.B, cr.bl, [1.0] * F, self.bins, blocks=self.blocks,
                              proposal_variances=proposal_variances, chain0=cr.chain,
                              n_iter_metropolis=self.n_iter)
        L = cr.L
        self._idx, self._valid = _unfold_index(self.spectra, self.bins, L, cr.device)
        self._lik = torch.zeros(cr.B, dtype=torch.float64, device=cr.device)
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
        self._acc = torch.zeros((cr.B, max(self.K * self.n_iter, 1)), dtype=torch.int32, device=cr.device)

    def _batched(self, binned_t):
        return binned_t if binned_t.dim() == 3 else binned_t[None]

    def unfold(self, binned_t):
        """utils.unfold_bins on the device: [B?, nspec, maxbins] -> [B?, nspec, L+1]."""
        out = _unfold_batch(self._batched(binned_t), self._idx, self._valid)
        return out if binned_t.dim() == 3 else out[0]

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
        """NonCenteredGibbs.py:333-355 (binned dict, dict / array map) -> float (B = 1)."""
        if self.cr.B != 1:
            raise NotImplementedError("compute_log_likelihood: the reference surface's one-chain form")
        bt = self.plan.dl_tensor(dls)[0]
        return float(self.loglik_t(self.unfold(bt), self.cr._s(s_nonCentered)).item())

    def sweep_t(self, s_nc, binned_t, iteration):
        """one sweep on device tensors, no host synchronisation: binned_t
        [B?, nspec, maxbins] -> (updated copy, accept flags [B?, K * n_iter] int32
        in decision order; the flags tensor is reused by the next sweep)."""
        plan, cr = self.plan, self.cr
        one = binned_t.dim() == 2
        dl = self._batched(binned_t).contiguous()
        if cr.rng == "replay":
            up, ua = plan.replay_mh_uniforms()
            prop, logr, _ = plan.mh_propose(dl, up, seed=cr.seed, iteration=iteration)
        else:
            prop, logr, ua = plan.mh_propose(dl, None, seed=cr.seed, iteration=iteration, with_uniforms=True)
        prop, logr = prop.contiguous(), logr.contiguous()
        cur = dl.clone()
        # every temporary stays referenced until the launch is enqueued (a freed
        # tensor's block is handed to the next allocation)
        dl_cur = _unfold_batch(cur, self._idx, self._valid)
        dl_prop = _unfold_batch(prop, self._idx, self._valid)
        u0 = ua.contiguous()
        _capi.check(self.cr.lib.gs_masked_pixel_mh(
            cr.handle, self.K, self.n_iter, plan.maxbins, _capi.ptr(self._blk), _capi.ptr(self._blk_lmax),
            _capi.ptr(self._blk_field), _capi.ptr(self._blk_bins), _capi.ptr(s_nc.contiguous()), _capi.ptr(dl_cur),
            _capi.ptr(dl_prop), _capi.ptr(logr), _capi.ptr(u0), _capi.ptr(prop),
            _capi.ptr(cur), _capi.ptr(self._acc), _capi.stream_ptr()), "gs_masked_pixel_mh")
        return (cur[0], self._acc[0]) if one else (cur, self._acc)

    def split_accept(self, flags):
        a = flags.cpu().numpy()
        out, off = {}, 0
        for s, n in self._acc_layout:
            out[s] = [int(v) for v in a[off:off + n]] if a.ndim == 1 else a[:, off:off + n].copy()
            off += n
        return out

    def sample_t(self, s_nc, binned_t, iteration):
        """one sweep on device tensors: binned_t [nspec, maxbins] (updated copy
        returned), s_nc [nspec, NR]; returns (binned_t, accept dict of lists)."""
        cur, flags = self.sweep_t(s_nc, binned_t, iteration)
        return cur, self.split_accept(flags)

    def sample(self, s_nonCentered, binned_dls_old, iteration=None):
        """reference surface: dict maps / binned dicts in, (binned dict, accept dict) out (B = 1)."""
        if self.cr.B != 1:
            raise NotImplementedError("PixelMH.sample: the reference surface's one-chain form (use sweep_t)")
        it = self.cr.iteration if iteration is None else int(iteration)
        bt = self.plan.dl_tensor(binned_dls_old)[0]
        cur, acc = self.sample_t(self.cr._s(s_nonCentered), bt, it)
        return self.plan.dl_dicts(cur[None])[0], acc


class MaskedMHRunner:
    """Masked non-centred and interweaving drivers (the context's B chains at once):

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
        """n_iter iterations from dls_init (binned dict, or a list of B dicts).
        s_init: continue from this map instead of the reference's PCG start map
        (ASIS.py:153-156).  The loop stays on the device (D_l, accept flags and
        histories are device tensors until the end; the stage times come from
        events read after it)."""
        cr, mh, plan = self.cr, self.mh, self.plan
        B = cr.B
        if isinstance(dls_init, (list, tuple)):
            init = [{s: np.asarray(d[s], dtype=np.float64) for s in mh.spectra} for d in dls_init]
        else:
            init = {s: np.asarray(dls_init[s], dtype=np.float64) for s in mh.spectra}
        cur = plan.dl_tensor(init)                             # [B, nspec, maxbins]
        shape = lambda t: t.reshape(cr._shape(*t.shape[1:])) if B == 1 else t
        hist, flags, acc_cr, evs = [cur], [], [], []
        dl = shape(mh.unfold(cur))
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
                dl = shape(mh.unfold(cur))
            else:
                if self.cr_kind == KIND_PCG:
                    s = self._pcg(dl, it)
                else:
                    cr.step(self.cr_kind, dl, s, iteration=it)
                    acc_cr.append(cr._acc.clone())
                ev[1].record()
                stats = plan.sweep_stats(self.d0[None], s.reshape(B, cr.F, cr.NR))
                var = plan.replay_invgamma() if cr.rng == "replay" else None
                tmp = plan.cls_draw(stats, var, seed=cr.seed, iteration=it)
                dl_tmp = shape(mh.unfold(tmp))
                s_nc = mh.noncentre(dl_tmp, s)
                ev[2].record()
                cur, f = mh.sweep_t(s_nc, tmp, it)
                dl = shape(mh.unfold(cur))
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
        H = torch.stack(hist).cpu().numpy()                   # [n_iter + 1, B, nspec, maxbins]
        one = B == 1
        h = {sp: (H[:, 0, k, :len(mh.bins[sp]) - 1] if one else H[:, :, k, :len(mh.bins[sp]) - 1]).copy()
             for k, sp in enumerate(mh.spectra)}
        acc = {sp: [] for sp in mh.spectra}
        if flags:
            Fl = torch.stack(flags).cpu().numpy().reshape(len(flags), B, -1)   # [n_iter, B, K n_iter]
            off = 0
            for sp, n in mh._acc_layout:
                a = Fl[:, :, off:off + n].astype(np.int64)
                acc[sp] = a[:, 0] if one else a
                off += n
        a_cr = torch.stack(acc_cr).cpu().numpy().astype(np.int64) if acc_cr else None
        if a_cr is not None and one:
            a_cr = a_cr[:, 0]
        out = (h, {sp: np.array(v) for sp, v in acc.items()})
        return out + (a_cr, t_it, t_cr, t_cls, t_nc)
