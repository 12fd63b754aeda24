"""Device-resident batched Gibbs engine over the HIP C-ABI.

One ``GibbsPlan`` holds a model (beam, noise, bins, MH blocks) on one GPU and
runs ``nchains`` independent chains in lock-step; every per-iteration array
stays in HBM (torch tensors used purely as device buffers) and each
iteration is a handful of asynchronous kernel launches on the current HIP
stream (capturable in a hipGraph).

RNG modes
  * ``native``: counter-based Philox streams on the device, keyed by
    (seed, global chain id) -- results do not depend on the GPU count.
  * ``replay``: numpy's legacy global RNG drawn on the host in the
    reference's exact order and uploaded, so a run reproduces
    the reference's numbers for the same ``np.random.seed``.
"""
import ctypes
import math

import numpy as np
import torch
from scipy.stats import invgamma

from . import _capi as C

SPECTRA = {1: ("TT",), 2: ("EE", "BB"), 3: ("TT", "EE", "BB", "TE")}
FIELDS = {1: ("TT",), 2: ("EE", "BB"), 3: ("TT", "EE", "BB")}
MH_ORDER = {1: ("TT",), 2: ("EE", "BB"), 3: ("EE", "BB", "TT", "TE")}


def _require_gpu():
    if not torch.cuda.is_available():
        raise C.GibbsHipError("gibbssampler_amd needs a ROCm GPU (MI355X); no CPU fallback")


class GibbsPlan:
    def __init__(self, lmax, nside, nfields, nchains, bl, noise_var, bins, blocks=None,
                 proposal_variances=None, chain0=0, quirks=C.GS_QUIRK_ASIS_RECENTRE_CENTERED,
                 n_iter_metropolis=1, device=None):
        _require_gpu()
        self.lib = C.load()
        self.L = int(lmax)
        self.nside = int(nside)
        self.Npix = 12 * self.nside ** 2
        self.F = int(nfields)
        self.nchains = int(nchains)
        self.chain0 = int(chain0)
        self.spectra = SPECTRA[self.F]
        self.fields = FIELDS[self.F]
        self.n_iter_metropolis = int(n_iter_metropolis)
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else
                                   torch.device(device).index or 0)
        self.bins = {s: np.asarray(bins[s], dtype=np.int32) for s in self.spectra}
        self.blocks = None if blocks is None else {s: np.asarray(blocks[s], dtype=np.int32) for s in self.spectra}
        self.proposal_variances = None if proposal_variances is None else \
            {s: np.asarray(proposal_variances[s], dtype=np.float64) for s in self.spectra}
        self.bl = np.ascontiguousarray(bl, dtype=np.float64)
        self.noise_var = np.ascontiguousarray(noise_var, dtype=np.float64)
        if self.bl.shape != (self.L + 1,):
            raise ValueError("bl must have lmax+1 entries")
        desc = C.GsModelDesc()
        desc.lmax, desc.nside, desc.nfields, desc.nchains = self.L, self.nside, self.F, self.nchains
        desc.chain0, desc.quirks, desc.n_iter_metropolis = self.chain0, int(quirks), self.n_iter_metropolis
        keep = [self.bl, self.noise_var]
        desc.bl = self.bl.ctypes.data_as(C.c_double_p)
        desc.noise_var = self.noise_var.ctypes.data_as(C.c_double_p)
        for k, s in enumerate(self.spectra):
            b = np.ascontiguousarray(self.bins[s], dtype=np.int32)
            keep.append(b)
            desc.bins[k] = b.ctypes.data_as(C.c_int_p)
            desc.nbin_edges[k] = len(b)
            if self.blocks is not None:
                bk = np.ascontiguousarray(self.blocks[s], dtype=np.int32)
                keep.append(bk)
                desc.blocks[k] = bk.ctypes.data_as(C.c_int_p)
                desc.nblock_edges[k] = len(bk)
            if self.proposal_variances is not None:
                pv = np.ascontiguousarray(self.proposal_variances[s], dtype=np.float64)
                if len(pv) != len(b) - 1 - 2:
                    raise ValueError(f"proposal_variances[{s}] must have nbins-2 entries")
                keep.append(pv)
                desc.prop_var[k] = pv.ctypes.data_as(C.c_double_p)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            C.check(self.lib.gs_plan_create(ctypes.byref(desc), ctypes.byref(h)), "gs_plan_create")
        self._h = h
        mb, ns, nacc, nsp = (ctypes.c_int() for _ in range(4))
        C.check(self.lib.gs_plan_info(h, ctypes.byref(mb), ctypes.byref(ns), ctypes.byref(nacc), ctypes.byref(nsp)))
        self.maxbins, self.nstat, self.nacc, self.nspec = mb.value, ns.value, nacc.value, nsp.value
        self.NR = (self.L + 1) ** 2
        nt, rpt = ctypes.c_int(), ctypes.c_int()
        C.check(self.lib.gs_plan_sweep_info(h, ctypes.byref(nt), ctypes.byref(rpt)))
        self.ntask, self.rows_per_task = nt.value, rpt.value
        # host-side replay helpers (data independent)
        ell = np.arange(self.L + 1, dtype=np.float64)
        expo = (2 * ell + 1) / 2
        self._alphas = {}
        for s in self.spectra:
            b = self.bins[s]
            a = np.array([np.sum(expo[b[i]:b[i + 1]]) - 1 for i in range(len(b) - 1)])
            a[0] = 1
            self._alphas[s] = a
        self._acc_layout = []
        if self.blocks is not None:
            for s in MH_ORDER[self.F]:
                self._acc_layout.append((s, (len(self.blocks[s]) - 1) * self.n_iter_metropolis))

    def __del__(self):
        try:
            C.park(dict(self.__dict__))       # inside a capture: tensors freed after it
            if getattr(self, "_h", None) is not None and self.lib is not None:
                C.release(self.lib.gs_plan_destroy, self._h)
                self._h = None
        except Exception:
            pass

    # ---- buffers ---------------------------------------------------------------
    def zeros(self, *shape, dtype=torch.float64):
        return torch.zeros(*shape, dtype=dtype, device=self.device)

    def dl_tensor(self, dls):
        """dict spec -> binned D (same for all chains) or list of dicts -> [nchains, nspec, maxbins]."""
        out = np.zeros((self.nchains, self.nspec, self.maxbins))
        per_chain = dls if isinstance(dls, (list, tuple)) else [dls] * self.nchains
        for c, d in enumerate(per_chain):
            for k, s in enumerate(self.spectra):
                v = np.asarray(d[s], dtype=np.float64)
                out[c, k, :len(v)] = v
        return torch.from_numpy(out).to(self.device)

    def dl_dicts(self, t):
        a = t.detach().cpu().numpy()
        return [{s: a[c, k, :len(self.bins[s]) - 1].copy() for k, s in enumerate(self.spectra)}
                for c in range(self.nchains)]

    def data_tensor(self, d_alm):
        """dict field -> real-layout alm (or array [F, NR]) -> device [F, NR]."""
        if isinstance(d_alm, dict):
            arr = np.stack([np.asarray(d_alm[f], dtype=np.float64) for f in self.fields])
        else:
            arr = np.asarray(d_alm, dtype=np.float64).reshape(self.F, self.NR)
        return torch.from_numpy(np.ascontiguousarray(arr)).to(self.device)

    def split_accept(self, acc):
        a = acc.detach().cpu().numpy()
        out, off = {}, 0
        for s, n in self._acc_layout:
            out[s] = a[:, off:off + n]
            off += n
        return out

    # ---- replay variates (numpy legacy global RNG, reference order) -------------
    def replay_cr_normals(self):
        z = np.stack([np.stack([np.random.normal(size=self.NR) for _ in range(self.F)])
                      for _ in range(self.nchains)])
        return torch.from_numpy(z).to(self.device)

    def replay_invgamma(self):
        v = np.zeros((self.nchains, self.nspec, self.maxbins))
        for c in range(self.nchains):
            for k, s in enumerate(self.spectra):
                x = invgamma.rvs(a=self._alphas[s])
                v[c, k, :len(x)] = x
        return torch.from_numpy(v).to(self.device)

    def replay_mh_uniforms(self):
        up = np.zeros((self.nchains, self.nspec, self.maxbins))
        ua = np.zeros((self.nchains, max(self.nacc, 1)))
        for c in range(self.nchains):
            for s in MH_ORDER[self.F]:
                k = self.spectra.index(s)
                nb = len(self.bins[s]) - 1
                up[c, k, 2:nb] = np.random.uniform(size=nb - 2)
            ua[c, :self.nacc] = np.random.uniform(size=self.nacc)
        return torch.from_numpy(up).to(self.device), torch.from_numpy(ua).to(self.device)

    # ---- stages ---------------------------------------------------------------
    def _s(self):
        return C.stream_ptr()

    def block_params(self, mode, dl, out=None):
        out = self.zeros(self.nchains, self.L + 1, C.GS_NPARAM) if out is None else out
        C.check(self.lib.gs_block_params(self._h, mode, C.ptr(dl), C.ptr(out), self._s()), "gs_block_params")
        return out

    def cr_sweep(self, d, params, z=None, seed=0, iteration=0, substep=0, s_out=None, store=True, stats=None):
        if store and s_out is None:
            s_out = self.zeros(self.nchains, self.F, self.NR)
        stats = self.zeros(self.nchains, self.nstat, self.L + 1) if stats is None else stats
        C.check(self.lib.gs_cr_sweep(self._h, C.ptr(d), C.ptr(params), C.ptr(z), int(seed), int(iteration),
                                     int(substep), C.ptr(s_out) if store else None, C.ptr(stats), self._s()),
                "gs_cr_sweep")
        return s_out, stats

    def sweep_stats(self, d, s, stats=None):
        """per-l statistics of a given map s [nchains, F, NR] (no draw)."""
        stats = self.zeros(self.nchains, self.nstat, self.L + 1) if stats is None else stats
        C.check(self.lib.gs_sweep_stats(self._h, C.ptr(d), C.ptr(s), C.ptr(stats), self._s()), "gs_sweep_stats")
        return stats

    def cls_draw(self, stats, variates=None, seed=0, iteration=0, out=None):
        out = self.zeros(self.nchains, self.nspec, self.maxbins) if out is None else out
        C.check(self.lib.gs_cls_draw(self._h, C.ptr(stats), C.ptr(variates), int(seed), int(iteration),
                                     C.ptr(out), self._s()), "gs_cls_draw")
        return out

    def mh_propose(self, dl, u_prop=None, seed=0, iteration=0, with_uniforms=False):
        """(prop, logr[, native accept uniforms]) of the NC MH step (no decisions)."""
        prop = self.zeros(self.nchains, self.nspec, self.maxbins)
        logr = self.zeros(self.nchains, self.nspec, self.maxbins)
        ua = self.zeros(self.nchains, max(self.nacc, 1)) if with_uniforms else None
        C.check(self.lib.gs_mh_propose(self._h, C.ptr(dl), C.ptr(u_prop), int(seed), int(iteration), C.ptr(prop),
                                       C.ptr(logr), C.ptr(ua), self._s()), "gs_mh_propose")
        return prop, logr, ua

    def nc_mh(self, stats, dl, u_prop=None, u_acc=None, seed=0, iteration=0, accept=None):
        accept = self.zeros(self.nchains, max(self.nacc, 1), dtype=torch.int32) if accept is None else accept
        C.check(self.lib.gs_nc_mh(self._h, C.ptr(stats), C.ptr(dl), C.ptr(u_prop), C.ptr(u_acc), int(seed),
                                  int(iteration), C.ptr(accept), self._s()), "gs_nc_mh")
        return accept

    def stats_to_noncentered(self, dl, stats):
        C.check(self.lib.gs_stats_to_noncentered(self._h, C.ptr(dl), C.ptr(stats), self._s()), "gs_stats_to_nc")
        return stats

    def recentre(self, dl_new, s, dl_old=None):
        C.check(self.lib.gs_recentre(self._h, C.ptr(dl_new), C.ptr(dl_old), C.ptr(s), self._s()), "gs_recentre")
        return s

    # ---- fused iterations -----------------------------------------------------------
    def step_centered(self, d, dl, s_out, z=None, igvar=None, seed=0, iteration=0):
        C.check(self.lib.gs_step_centered(self._h, C.ptr(d), C.ptr(dl), C.ptr(s_out), C.ptr(z), C.ptr(igvar),
                                          int(seed), int(iteration), self._s()), "gs_step_centered")

    def step_centered_fused(self, d, dl, s_out, seed=0, iteration=0, trace=None, capacity=0):
        """gs_step_centered with the trace record and device-counter advance in the
        C_l-draw launch (graph-captured native steps)."""
        C.check(self.lib.gs_step_centered_fused(self._h, C.ptr(d), C.ptr(dl), C.ptr(s_out), int(seed), int(iteration),
                                                C.ptr(trace), int(capacity), self._s()), "gs_step_centered_fused")

    def step_asis_fused(self, d, dl, s_out, seed=0, iteration=0, accept=None, dl_tmp=None, recentre=False,
                        trace=None, capacity=0):
        """gs_step_asis with the trace record and device-counter advance in the MH launch."""
        C.check(self.lib.gs_step_asis_fused(self._h, C.ptr(d), C.ptr(dl), C.ptr(s_out), int(seed), int(iteration),
                                            C.ptr(accept), C.ptr(dl_tmp), 1 if recentre else 0, C.ptr(trace),
                                            int(capacity), self._s()), "gs_step_asis_fused")

    def step_noncentered(self, d, dl, s_out, z=None, u_prop=None, u_acc=None, seed=0, iteration=0, accept=None):
        C.check(self.lib.gs_step_noncentered(self._h, C.ptr(d), C.ptr(dl), C.ptr(s_out), C.ptr(z), C.ptr(u_prop),
                                             C.ptr(u_acc), int(seed), int(iteration), C.ptr(accept), self._s()),
                "gs_step_noncentered")

    # the three stages of step_noncentered (for pipelined schedules)
    def nc_prologue(self, dl, u_prop=None, seed=0, iteration=0):
        C.check(self.lib.gs_nc_prologue(self._h, C.ptr(dl), C.ptr(u_prop), int(seed), int(iteration), self._s()),
                "gs_nc_prologue")

    def nc_sweep(self, d, dl, s_out, z=None, seed=0, iteration=0, finish=True):
        C.check(self.lib.gs_nc_sweep(self._h, C.ptr(d), C.ptr(dl), C.ptr(s_out), C.ptr(z), int(seed), int(iteration),
                                     int(bool(finish)), self._s()), "gs_nc_sweep")

    def nc_finish(self):
        C.check(self.lib.gs_nc_finish(self._h, self._s()), "gs_nc_finish")

    def nc_decide(self, dl, u_acc=None, seed=0, iteration=0, accept=None):
        C.check(self.lib.gs_nc_decide(self._h, C.ptr(dl), C.ptr(u_acc), int(seed), int(iteration), C.ptr(accept),
                                      self._s()), "gs_nc_decide")

    def nc_decide_fused(self, dl, seed=0, iteration=0, accept=None, trace=None, capacity=0):
        C.check(self.lib.gs_nc_decide_fused(self._h, C.ptr(dl), int(seed), int(iteration), C.ptr(accept),
                                            C.ptr(trace), int(capacity), self._s()), "gs_nc_decide_fused")

    def step_asis(self, d, dl, s_out, z=None, igvar=None, u_prop=None, u_acc=None, seed=0, iteration=0,
                  accept=None, dl_tmp=None, recentre=False):
        C.check(self.lib.gs_step_asis(self._h, C.ptr(d), C.ptr(dl), C.ptr(s_out), C.ptr(z), C.ptr(igvar),
                                      C.ptr(u_prop), C.ptr(u_acc), int(seed), int(iteration), C.ptr(accept),
                                      C.ptr(dl_tmp), 1 if recentre else 0, self._s()), "gs_step_asis")

    # ---- hipGraph support ---------------------------------------------------------------
    def iteration_counter(self, enable, start=1):
        C.check(self.lib.gs_iteration_counter(self._h, 1 if enable else 0, int(start)), "gs_iteration_counter")

    def graph_step(self, offset, advance):
        """Offset of the next captured step from the device base, and the advance
        its last launch applies (gs_graph_step)."""
        C.check(self.lib.gs_graph_step(self._h, int(offset), int(advance)), "gs_graph_step")

    def advance_iteration(self):
        C.check(self.lib.gs_advance_iteration(self._h, self._s()), "gs_advance_iteration")

    def record_trace(self, dl, trace, capacity, iteration=0):
        C.check(self.lib.gs_record_trace(self._h, C.ptr(dl), C.ptr(trace), int(capacity), int(iteration), self._s()),
                "gs_record_trace")

    # ---- timing of the dominant kernel (hipEvents on the launch stream) ---------------
    def sweep_timing(self, enable):
        """True: start bracketing every CR sweep with hipEvents; False: stop and
        return (total ms, launches); "pause" / "resume" keep the launches timed so far."""
        mode = {True: 1, False: 0, "pause": 2, "resume": 3}[enable]
        tot = ctypes.c_double()
        n = ctypes.c_int()
        C.check(self.lib.gs_sweep_timing(self._h, mode, ctypes.byref(tot), ctypes.byref(n)))
        return tot.value, n.value


def stats_layout(F):
    """Names of the statistic rows (include/gibbs_capi.h GS_NSTAT_*)."""
    return {1: ["ssTT", "dTsT"], 2: ["ssEE", "ssBB", "dEsE", "dBsB"],
            3: ["ssTT", "ssEE", "ssBB", "ssTE", "dTsT", "dEsT", "dEsE", "dBsB"]}[F]

