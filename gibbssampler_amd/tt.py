"""Temperature-only samplers and drivers from pixel data.

The reference's TT path (HEAD) works on the T map with healpy transforms:

  CenteredConstrainedRealization     CenteredGibbs.py:103-236
    sample_no_mask (full sky)        108-132   -> gs_masked_tt_fullsky (centred)
    sample_mask (qcinv PCG)          135-191   -> gs_masked_pcg_rhs / _pcg_solve
    sample_gibbs_change_variable     193-213   -> gs_masked_cr(GS_MCR_AUX), n_gibbs 1
  NonCenteredConstrainedRealization  NonCenteredGibbs.py:17-101
    sample_no_mask                   22-38     -> gs_masked_tt_fullsky (non-centred)
    sample_mask (qcinv, C^-1/2 out)  41-92     -> PCG, then C^-1/2 (gs_masked_center)
  CenteredClsSampler.sample          CenteredGibbs.py:21-48  -> gs_sweep_stats + gs_cls_draw
  NonCenteredClsSampler.sample       NonCenteredGibbs.py:212-249, likelihood
                                     ClsSampler.py:96-109    -> masked.PixelMH (F = 1)
  drivers: GibbsSampler.run_temperature (GibbsSampler.py:76-116),
           NonCenteredClsSampler... NonCenteredGibbs.run_temperature (488-527),
           MHClsSampler... ASIS.run_temperature (ASIS.py:69-131)

HEAD cannot run this path as shipped: ``config.mask_inversion``
is missing, ``config.bins`` is the polarization dict, ``utils.synthesis_hp`` does
not exist.  This module implements the intended semantics (mask_inversion =
the l < 2 slots, the sampler's own TT bins, synthesis_hp = alm2map of the real
layout); the fixtures of tools/gen_golden_tt.py run the reference with exactly
those three fixes, so replay-mode results here match the reference's numbers.

State stays on the device between steps; the reference-surface classes move
numpy arrays in and out like the reference's.  Replay mode draws numpy's
global stream in the reference's order; native mode uses the Philox streams.
"""
import time

import numpy as np
import torch

from . import _capi
from .masked import MaskedCR, PixelMH, KIND_PCG


def _dl_from_var(var_cls, L):
    """per-slot variance (utils.generate_var_cl) -> unbinned D_l: var at the m = 0
    slot l is C_l; D_l = C_l l(l+1)/2pi (D_0 = var_0, utils.py:126-129)."""
    v = np.asarray(var_cls, dtype=np.float64)[:L + 1]
    ell = np.arange(L + 1, dtype=np.float64)
    return np.where(ell > 0, v * ell * (ell + 1) / (2 * np.pi), v)


class TTModel:
    """Device context of the TT chains: the masked-CR context (F = 1), the
    C_l-draw plan and (for non-centred / ASIS runs) the pixel-likelihood MH.
    ``nchains`` = B > 1 runs B chains (global ids chain .. chain + B - 1) as one
    batch (batched SHTs); the drivers' histories then carry a chain axis."""

    def __init__(self, pix_map, noise, bl, lmax, nside, bins, mask=None, blocks=None, proposal_variances=None,
                 n_iter_metropolis=1, rng="native", seed=0, chain=0, pcg_accuracy=1.0e-6, nchains=1,
                 sht_mode="auto"):
        from .engine import GibbsPlan
        self.L, self.nside = int(lmax), int(nside)
        self.NR = (self.L + 1) ** 2
        self.bins = np.asarray(bins)
        self.B = int(nchains)
        # TT PCG: 1e-6 relative, 4000 iterations (ConstrainedRealization.py:41)
        self.cr = MaskedCR(pix_map, noise, 1.0, bl, lmax, nside, mask=mask, nfields=1, gibbs_cr=True, n_gibbs=1,
                           rng=rng, seed=seed, chain=chain, pcg_accuracy=pcg_accuracy, nchains=self.B,
                           sht_mode=sht_mode)
        self.masked = mask is not None
        self.rng, self.seed = rng, int(seed)
        self.plan = GibbsPlan(lmax, nside, 1, self.B, self.cr.bl, [1.0], {"TT": self.bins}, chain0=chain)
        self.d0 = self.plan.zeros(1, 1, self.NR)
        self.mh = None
        if proposal_variances is not None:
            nb = len(self.bins) - 1
            blk = np.asarray(blocks) if blocks is not None else np.arange(2, nb + 1)   # ClsSampler.py:64-65
            self.mh = PixelMH(self.cr, {"TT": self.bins}, {"TT": blk},
                              {"TT": np.asarray(proposal_variances, dtype=np.float64)}, n_iter_metropolis)
        idx = np.full((1, self.L + 1), -1, dtype=np.int64)
        for i in range(len(self.bins) - 1):
            idx[0, self.bins[i]:min(self.bins[i + 1], self.L + 1)] = i
        self._idx = torch.from_numpy(np.maximum(idx, 0)).to(self.cr.device)
        self._valid = torch.from_numpy(idx >= 0).to(self.cr.device)

    # -- device steps --------------------------------------------------------------------
    def unfold(self, binned_t):
        """[B?, 1, maxbins] binned D -> [B?, 1, L+1] (utils.unfold_bins)."""
        if binned_t.dim() == 2:
            return torch.where(self._valid, torch.gather(binned_t, 1, self._idx), 0.0).contiguous()
        B = binned_t.shape[0]
        g = torch.gather(binned_t, 2, self._idx.unsqueeze(0).expand(B, -1, -1))
        return torch.where(self._valid.unsqueeze(0), g, 0.0).contiguous()

    def binned_t(self, binned):
        """binned D_l (one array for every chain, or [B, nbins]) -> [1, maxbins] (B = 1) / [B, 1, maxbins]"""
        a = np.asarray(binned, dtype=np.float64)
        t = self.plan.dl_tensor([{"TT": r} for r in a] if a.ndim == 2 else {"TT": a})
        return t[0] if self.B == 1 else t

    def cr_centered(self, dl, it):
        """sample_no_mask (full sky) or sample_mask (PCG) in the centred parametrisation."""
        if self.masked:
            return self.cr.pcg_solve(dl, self.cr.pcg_rhs(dl, iteration=it))
        return self.cr.tt_fullsky(dl, noncentered=False, iteration=it)

    def cr_noncentered(self, dl, it):
        if self.masked:
            return self.centre(dl, self.cr.pcg_solve(dl, self.cr.pcg_rhs(dl, iteration=it)), -1)
        return self.cr.tt_fullsky(dl, noncentered=True, iteration=it)

    def cr_aux(self, dl, s, it):
        """sample_gibbs_change_variable: one v | s, s | v pass (in place)."""
        self.cr.step(_capi.GS_MCR_AUX, dl, s, iteration=it)
        return s

    def centre(self, dl, s, direction):
        out = torch.empty_like(s)
        _capi.check(self.cr.lib.gs_masked_center(self.cr.handle, _capi.ptr(dl), int(direction), _capi.ptr(s),
                                                 _capi.ptr(out), _capi.stream_ptr()), "gs_masked_center")
        return out

    def cls_draw(self, s, it):
        stats = self.plan.sweep_stats(self.d0, s.reshape(self.B, 1, self.NR))
        var = self.plan.replay_invgamma() if self.rng == "replay" else None
        out = self.plan.cls_draw(stats, var, seed=self.seed, iteration=it)
        return out[0] if self.B == 1 else out

    def mh_sweep(self, s_nc, binned_t, it):
        cur, acc = self.mh.sample_t(s_nc, binned_t, it)
        return cur, acc["TT"]

    def host_binned(self, t):
        if self.B == 1:
            return t[0, :len(self.bins) - 1].cpu().numpy().copy()
        return t[:, 0, :len(self.bins) - 1].cpu().numpy().copy()

    def _start(self, dls_init):
        a = np.asarray(dls_init, dtype=np.float64).copy()
        return a if self.B == 1 or a.ndim == 2 else np.broadcast_to(a, (self.B,) + a.shape).copy()

    def _ones(self):
        return 1 if self.B == 1 else np.ones(self.B, dtype=np.int64)

    # -- drivers -------------------------------------------------------------------------
    def run_centered(self, dls_init, n_iter):
        """GibbsSampler.run_temperature (GibbsSampler.py:76-116)."""
        cur = self.binned_t(dls_init)
        dl = self.unfold(cur)
        s = self.cr_centered(dl, 0)                  # the first CR (GibbsSampler.py:92)
        h, acc, t = [self._start(dls_init)], [], []
        for i in range(n_iter):
            t0 = time.perf_counter()
            s = self.cr_centered(dl, i + 1)
            cur = self.cls_draw(s, i + 1)
            dl = self.unfold(cur)
            acc.append(self._ones())
            h.append(self.host_binned(cur))
            t.append(time.perf_counter() - t0)
        self.s = s
        return np.array(h), np.array(acc), t

    def run_noncentered(self, dls_init, n_iter):
        """NonCenteredGibbs.run_temperature (NonCenteredGibbs.py:488-527): no
        initial entry in the history (the reference appends after each step)."""
        cur = self.binned_t(dls_init)
        dl = self.unfold(cur)
        h, acc, t = [], [], []
        for i in range(n_iter):
            t0 = time.perf_counter()
            s_nc = self.cr_noncentered(dl, i + 1)
            cur, a = self.mh_sweep(s_nc, cur, i + 1)
            dl = self.unfold(cur)
            acc.append(a)
            h.append(self.host_binned(cur))
            t.append(time.perf_counter() - t0)
        self.s = s_nc
        return np.array(h), np.array(acc), np.array(t)

    def run_asis(self, dls_init, n_iter, gibbs_cr=False):
        """MHClsSampler... ASIS.run_temperature (ASIS.py:69-131); re-centring with
        s_nc (ASIS.py:120, correct in the TT path)."""
        cur = self.binned_t(dls_init)
        dl = self.unfold(cur)
        s = self.cr_centered(dl, 0)                  # ASIS.py:87
        h, acc, acc_cr, t = [self._start(dls_init)], [], [], []
        for i in range(n_iter):
            it = i + 1
            t0 = time.perf_counter()
            if gibbs_cr:
                s = self.cr_aux(dl, s, it)
            else:
                s = self.cr_centered(dl, it)
            acc_cr.append(self._ones())
            tmp = self.cls_draw(s, it)
            s_nc = self.centre(self.unfold(tmp), s, -1)
            cur, a = self.mh_sweep(s_nc, tmp, it)
            dl = self.unfold(cur)
            s = self.centre(dl, s_nc, +1)
            acc.append(a)
            h.append(self.host_binned(cur))
            t.append(time.perf_counter() - t0)
        self.s = s
        return np.array(h), np.array(acc), np.array(acc_cr), np.array(t)


# ---------------------------------------------------------------------------------------
# reference-surface step objects (numpy in / numpy out)
# ---------------------------------------------------------------------------------------
class TTCenteredConstrainedRealization:
    """CenteredConstrainedRealization (CenteredGibbs.py:103-236)."""

    def __init__(self, model):
        self.model = model
        self.cr = model.cr
        self.mask_path = "mask" if model.masked else None

    def _dl(self, var_cls):
        return torch.from_numpy(_dl_from_var(var_cls, self.model.L)[None].copy()).to(self.cr.device)

    def _s(self, s):
        return torch.from_numpy(np.ascontiguousarray(s, dtype=np.float64).reshape(1, -1).copy()).to(self.cr.device)

    def sample_no_mask(self, var_cls):
        return self.cr.tt_fullsky(self._dl(var_cls), noncentered=False)[0].cpu().numpy(), 1

    def sample_mask(self, cls_, var_cls, s_old, metropolis_step=False):
        if metropolis_step:
            raise NotImplementedError("RJPO (metropolis_step) is not reachable from HEAD's drivers")
        dl = self._dl(var_cls)
        return self.cr.pcg_solve(dl, self.cr.pcg_rhs(dl))[0].cpu().numpy(), 1

    def sample_gibbs_change_variable(self, var_cls, old_s):
        s = self._s(old_s)
        self.cr.step(_capi.GS_MCR_AUX, self._dl(var_cls), s)
        return s[0].cpu().numpy(), 1

    def sample(self, cls_, var_cls, old_s, metropolis_step=False, use_gibbs=False):
        if use_gibbs:
            return self.sample_gibbs_change_variable(var_cls, old_s)
        if self.mask_path is not None:
            return self.sample_mask(cls_, var_cls, old_s, metropolis_step)
        return self.sample_no_mask(var_cls)


class TTNonCenteredConstrainedRealization(TTCenteredConstrainedRealization):
    """NonCenteredConstrainedRealization (NonCenteredGibbs.py:17-101)."""

    def sample_no_mask(self, cls_, var_cls):
        return self.cr.tt_fullsky(self._dl(var_cls), noncentered=True)[0].cpu().numpy(), 1

    def sample_mask(self, cls_, var_cls, s_old, metropolis_step=False):
        if metropolis_step:
            raise NotImplementedError("RJPO (metropolis_step) is not reachable from HEAD's drivers")
        dl = self._dl(var_cls)
        return self.model.centre(dl, self.cr.pcg_solve(dl, self.cr.pcg_rhs(dl)), -1)[0].cpu().numpy(), 1

    def sample(self, cls_, var_cls, old_s, metropolis_step=False):
        if self.mask_path is not None:
            return self.sample_mask(cls_, var_cls, old_s, metropolis_step)
        return self.sample_no_mask(cls_, var_cls)


class TTCenteredClsSampler:
    """CenteredClsSampler.sample (CenteredGibbs.py:24-48): binned D_l."""

    def __init__(self, model):
        self.model = model

    def sample(self, alms):
        s = torch.from_numpy(np.ascontiguousarray(alms, dtype=np.float64).reshape(1, -1).copy()).to(
            self.model.cr.device)
        return self.model.host_binned(self.model.cls_draw(s, self.model.cr.iteration))


class TTNonCenteredClsSampler:
    """NonCenteredClsSampler.sample (NonCenteredGibbs.py:212-249): returns
    (binned D_l, per-slot variance of it, accept list)."""

    def __init__(self, model):
        self.model = model

    def compute_log_likelihood(self, var_cls, s_nonCentered):
        m = self.model
        dl = torch.from_numpy(_dl_from_var(var_cls, m.L)[None].copy()).to(m.cr.device)
        s = torch.from_numpy(np.ascontiguousarray(s_nonCentered, dtype=np.float64).reshape(1, -1).copy()).to(
            m.cr.device)
        return float(m.mh.loglik_t(dl, s).item())

    def sample(self, s_nonCentered, binned_dls_old, var_cls_old=None):
        from .utils import generate_var_cl, unfold_bins
        m = self.model
        s = torch.from_numpy(np.ascontiguousarray(s_nonCentered, dtype=np.float64).reshape(1, -1).copy()).to(
            m.cr.device)
        cur, acc = m.mh_sweep(s, m.binned_t(binned_dls_old), m.cr.iteration)
        b = m.host_binned(cur)
        return b, generate_var_cl(unfold_bins(b, m.bins)), acc
