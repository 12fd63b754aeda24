"""Batched full-sky Gibbs drivers on the device (the loops of the reference drivers).

``BatchedRunner`` runs ``nchains`` chains of one of the three samplers in
lock-step on one GPU:

  * ``centered``    GibbsSampler.run_polarization (GibbsSampler.py:118-180): an
                    initial CR (ula=True, GibbsSampler.py:41,136-138), then per
                    iteration CR (closed form, CenteredGibbs.py:317-353 -- the
                    exact full-sky limit of the PCG branch) + inverse-Gamma /
                    inverse-Wishart C_l draw.  History includes the start.
  * ``noncentered`` NonCenteredGibbs.run_polarization (NonCenteredGibbs.py:529-571),
                    all_sph: non-centered CR + MH blocks.  History includes the start.
  * ``asis``        ASIS.run_polarization (ASIS.py:134-226): centered CR, centered
                    C_l draw, non-centering, NC MH, re-centring.  History
                    excludes the start (ASIS.py:150-206).

Everything stays in HBM; only the returned histories are copied back.
"""
import contextlib
import gc
import time

import numpy as np
import torch

from . import _capi as C
from .engine import GibbsPlan, MH_ORDER

INIT_ITER = 0xFFFFFFFF


@contextlib.contextmanager
def _capture(g):
    """torch.cuda.graph(g), capture-safe for other objects' teardown:
    - the cyclic collector is paused from before the capture opens until after
      it has closed (torch.cuda.graph's own gc.collect() in __enter__ still runs:
      an explicit collect ignores gc.disable);
    - any destructor that does run inside (a plain refcount drop in the
      captured code, or an explicit gc.collect()) parks its device resources
      in _capi's graveyard instead of calling HIP; they are released after the
      capture (_capi.end_capture)."""
    was = gc.isenabled()
    gc.disable()
    C.begin_capture()
    try:
        with torch.cuda.graph(g):
            yield
    finally:
        C.end_capture()
        if was:
            gc.enable()


class BatchedRunner:
    def __init__(self, kind, lmax, nside, nfields, nchains, bl, noise_var, bins, d_alm, blocks=None,
                 proposal_variances=None, rng="native", seed=0, chain0=0, quirks=1, n_iter_metropolis=1,
                 materialize_recentre=False, store_skymap=True):
        if kind not in ("centered", "noncentered", "asis"):
            raise ValueError(kind)
        if rng not in ("native", "replay"):
            raise ValueError(rng)
        self.kind, self.rng, self.seed = kind, rng, int(seed)
        self.quirks = int(quirks)
        self.plan = GibbsPlan(lmax, nside, nfields, nchains, bl, noise_var, bins, blocks=blocks,
                              proposal_variances=proposal_variances, chain0=chain0, quirks=quirks,
                              n_iter_metropolis=n_iter_metropolis)
        p = self.plan
        self.d = p.data_tensor(d_alm)
        self.s = p.zeros(p.nchains, p.F, p.NR) if store_skymap else None
        self.dl = None
        self.dl_tmp = p.zeros(p.nchains, p.nspec, p.maxbins)
        self.accept = p.zeros(p.nchains, max(p.nacc, 1), dtype=torch.int32)
        self.materialize_recentre = materialize_recentre
        self.iteration = 0
        self.graph = None

    def __del__(self):
        # dropped inside another sampler's capture: keep the kept hipGraphs, the
        # copy stream and the tensors alive until that capture has ended
        # (their destructors call HIP, which is illegal while a capture is open)
        try:
            C.park(dict(self.__dict__))
        except Exception:
            pass

    # -- one iteration ---------------------------------------------------------------
    def _replay(self):
        p = self.plan
        z = p.replay_cr_normals()
        ig = up = ua = None
        if self.kind in ("centered", "asis"):
            ig = p.replay_invgamma()
        if self.kind in ("noncentered", "asis"):
            up, ua = p.replay_mh_uniforms()
        return z, ig, up, ua

    def init(self, dls_init):
        p = self.plan
        if self.dl is None:
            self.dl = p.dl_tensor(dls_init)
        else:
            # keep the buffer a captured graph points at; a re-init drops the graph
            # (its device iteration counter belongs to the previous run)
            self.dl.copy_(p.dl_tensor(dls_init))
        self.graph = None
        p.iteration_counter(False)
        self.iteration = 0
        if self.kind == "centered":
            # the reference's initial CR (GibbsSampler.py:136-138) -- consumes its draws
            z = p.replay_cr_normals() if self.rng == "replay" else None
            params = p.block_params(0, self.dl)
            p.cr_sweep(self.d, params, z=z, seed=self.seed, iteration=INIT_ITER, s_out=self.s,
                       store=self.s is not None)

    # -- checkpoint / resume -----------------------------------------------------------
    def state_dict(self):
        """The chains' whole state between iterations, as host tensors and plain
        values (``torch.save`` / ``torch.load(weights_only=True)`` round-trip it):
        D_l, the last accept flags, ASIS's D_l before the MH, the sky map when
        stored, and the iteration count.  The native streams are counter-based
        (seed, chain id, iteration), so a restored runner continues the same
        trajectory bit for bit.  Replay runs draw from numpy's global RNG: its
        state is saved too (``numpy_rng_*``) and restored by load_state_dict."""
        if self.dl is None:
            raise RuntimeError("state_dict: the runner has not been initialised (run() or init() first)")
        p = self.plan
        st = {"kind": self.kind, "rng": self.rng, "seed": self.seed, "iteration": int(self.iteration),
              "chain0": p.chain0, "nchains": p.nchains, "lmax": p.L, "nfields": p.F,
              "dl": self.dl.cpu().clone(), "dl_tmp": self.dl_tmp.cpu().clone(), "accept": self.accept.cpu().clone(),
              "s": None if self.s is None else self.s.cpu().clone()}
        if self.rng == "replay":
            name, keys, pos, has_gauss, cached = np.random.get_state()
            st.update(numpy_rng_keys=torch.from_numpy(np.asarray(keys, dtype=np.int64)), numpy_rng_pos=int(pos),
                      numpy_rng_has_gauss=int(has_gauss), numpy_rng_cached=float(cached))
        return st

    def load_state_dict(self, st):
        """Restore a state_dict() (same kind, chains, l_max, fields and RNG mode);
        the device buffers are kept (a kept graph still points at them)."""
        p = self.plan
        want = {"kind": self.kind, "rng": self.rng, "chain0": p.chain0, "nchains": p.nchains, "lmax": p.L,
                "nfields": p.F}
        bad = {k: (st.get(k), v) for k, v in want.items() if st.get(k) != v}
        if bad:
            raise ValueError(f"load_state_dict: state does not match this runner: {bad}")
        dl = st["dl"].to(self.dl_tmp.device)
        if self.dl is None:
            self.dl = dl.clone()
        else:
            self.dl.copy_(dl)
        self.dl_tmp.copy_(st["dl_tmp"])
        self.accept.copy_(st["accept"])
        if self.s is not None and st.get("s") is not None:
            self.s.copy_(st["s"])
        if int(st["seed"]) != self.seed:
            # the kept chunk graphs of run() hold the old seed as a kernel
            # argument: drop them, so the resumed run captures with the new one
            self.__dict__.pop("_run_graphs", None)
        self.seed = int(st["seed"])
        self.iteration = int(st["iteration"])
        self.graph = None
        p.iteration_counter(False)
        if self.rng == "replay" and "numpy_rng_keys" in st:
            np.random.set_state(("MT19937", st["numpy_rng_keys"].numpy().astype(np.uint32), st["numpy_rng_pos"],
                                 st["numpy_rng_has_gauss"], st["numpy_rng_cached"]))

    # -- hipGraph: capture one whole iteration, replay it per step ------------------
    def capture_graph(self, trace=None, trace_capacity=None):
        """Capture one iteration (plus an optional device-side trace record) in a
        hipGraph; subsequent ``step()`` calls replay it.  Native RNG only: the
        iteration counter lives on the device and advances inside the graph."""
        if self.rng != "native":
            raise ValueError("graph capture needs the native (counter-based) RNG")
        p = self.plan
        p.iteration_counter(True, self.iteration + 1)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with _capture(g):
            if self.kind == "noncentered":
                # NC: prologue, sweep (+ statistics), MH decisions with the trace record
                # and the counter advance fused into the decision launch
                p.nc_prologue(self.dl, seed=self.seed)
                p.nc_sweep(self.d, self.dl, self.s, seed=self.seed)
                p.nc_decide_fused(self.dl, seed=self.seed, accept=self.accept, trace=trace,
                                  capacity=trace_capacity or 0)
            elif self.kind == "centered":
                # centered: the trace record and the counter advance ride in the C_l draw
                p.step_centered_fused(self.d, self.dl, self.s, seed=self.seed, trace=trace,
                                      capacity=trace_capacity or 0)
            else:
                # ASIS: the trace record and the counter advance ride in the MH launch
                p.step_asis_fused(self.d, self.dl, self.s, seed=self.seed, accept=self.accept, dl_tmp=self.dl_tmp,
                                  recentre=self.materialize_recentre, trace=trace, capacity=trace_capacity or 0)
        self.graph = g
        self.graph_steps = 1
        return g

    def capture_steps(self, nsteps, trace=None, trace_capacity=None, time_sweeps=False, time_every=1,
                      accept_trace=None):
        """Native RNG: capture ``nsteps`` whole iterations in ONE hipGraph (one
        replay = nsteps steps).  time_sweeps: bracket the CR-sweep kernel of every
        ``time_every``-th step by event-record nodes (plan.sweep_timing), so the
        sweep's duration is measured on its own stream inside the replay (an event
        node costs ~5 us of the step); collect with plan.sweep_timing(False)."""
        if self.rng != "native":
            raise ValueError("capture_steps: native RNG runs only")
        p = self.plan
        p.iteration_counter(True, self.iteration + 1)
        torch.cuda.synchronize()
        if time_sweeps:
            p.sweep_timing(True)
        g = torch.cuda.CUDAGraph()
        try:
            with _capture(g):
                for i in range(nsteps):
                    # step i reads base + i; only the last step's last launch advances
                    # the base (by nsteps): one counter ticket per replay
                    p.graph_step(i, nsteps if i == nsteps - 1 else 0)
                    if time_sweeps:
                        p.sweep_timing("resume" if i % time_every == 0 else "pause")
                    # accept_trace [nsteps, nchains, nacc]: step i writes its own slot
                    acc = self.accept if accept_trace is None else accept_trace[i]
                    if self.kind == "noncentered":
                        p.nc_prologue(self.dl, seed=self.seed)
                        p.nc_sweep(self.d, self.dl, self.s, seed=self.seed, finish=False)
                        p.nc_finish()
                        p.nc_decide_fused(self.dl, seed=self.seed, accept=acc, trace=trace,
                                          capacity=trace_capacity or 0)
                    elif self.kind == "centered":
                        p.step_centered_fused(self.d, self.dl, self.s, seed=self.seed, trace=trace,
                                              capacity=trace_capacity or 0)
                    else:
                        p.step_asis_fused(self.d, self.dl, self.s, seed=self.seed, accept=acc,
                                          dl_tmp=self.dl_tmp, recentre=self.materialize_recentre, trace=trace,
                                          capacity=trace_capacity or 0)
        finally:
            # back to one step per replay even when a launch raised inside the capture
            p.graph_step(0, 1)
        self.graph = g
        self.graph_steps = nsteps
        return g

    def _launch_step(self, it, z=None, ig=None, up=None, ua=None):
        p = self.plan
        if self.kind == "centered":
            p.step_centered(self.d, self.dl, self.s, z=z, igvar=ig, seed=self.seed, iteration=it)
        elif self.kind == "noncentered":
            p.step_noncentered(self.d, self.dl, self.s, z=z, u_prop=up, u_acc=ua, seed=self.seed, iteration=it,
                               accept=self.accept)
        else:
            p.step_asis(self.d, self.dl, self.s, z=z, igvar=ig, u_prop=up, u_acc=ua, seed=self.seed, iteration=it,
                        accept=self.accept, dl_tmp=self.dl_tmp, recentre=self.materialize_recentre)

    def step(self):
        if getattr(self, "graph", None) is not None:
            self.graph.replay()
            self.iteration += getattr(self, "graph_steps", 1)
            return
        p = self.plan
        it = self.iteration + 1
        z = ig = up = ua = None
        if self.rng == "replay":
            z, ig, up, ua = self._replay()
        self._launch_step(it, z, ig, up, ua)
        self.iteration = it

    # -- a whole run --------------------------------------------------------------------
    def run(self, dls_init, n_iter, timings=False, gather=None, graph_chunk=32, resume=None):
        """n_iter iterations from dls_init; returns (histories, accepts[, step
        times]).  gather: ShardContext.gather of a torchrun job -- the device
        histories of every rank are all-gathered along the chain axis (global
        chain order) before the one copy to the host.  resume: a state_dict()
        to continue from instead of starting at dls_init (the history's first
        row is then the restored D_l, i.e. the previous run's last row)."""
        p = self.plan
        if resume is not None:
            self.load_state_dict(resume)
        else:
            self.init(dls_init)
        with_start = self.kind != "asis"
        H = p.zeros(n_iter + (1 if with_start else 0), p.nchains, p.nspec, p.maxbins)
        A = p.zeros(n_iter, p.nchains, max(p.nacc, 1), dtype=torch.int32)
        if with_start:
            H[0].copy_(self.dl)
        t_steps = []
        if self.rng == "native" and graph_chunk and n_iter > 0:
            # the iterations as replays of captured hipGraphs of `chunk` steps
            # (device-side D_l / accept traces, no host synchronisation inside a
            # chunk); step times = chunk time / steps from events on the stream.
            # The graphs (and the trace buffers they write) are kept per chunk
            # length across run() calls: a later run replays them without
            # capturing again (the device counter base is set before each run)
            chunk = min(int(graph_chunk), n_iter)
            off = 1 if with_start else 0
            cache = self.__dict__.setdefault("_run_graphs", {})
            if cache.get("chunk") != chunk:
                cache.clear()
                cache["chunk"] = chunk
                cache["trace"] = p.zeros(chunk, p.nchains, p.nspec, p.maxbins)
                cache["acc"] = p.zeros(chunk, p.nchains, max(p.nacc, 1), dtype=torch.int32)
            trace, acc_tr = cache["trace"], cache["acc"]
            # single-rank runs: each finished chunk of the histories goes to pinned
            # host memory on a copy stream while the next chunk computes (only the
            # last chunk's transfer is left after the loop)
            if gather is None:
                Hh = torch.empty(H.shape, dtype=H.dtype, pin_memory=True)
                Ah = torch.empty(A.shape, dtype=A.dtype, pin_memory=True)
                cs = cache.setdefault("copy_stream", torch.cuda.Stream())
            p.iteration_counter(True, self.iteration + 1)
            done = 0
            while done < n_iter:
                k = min(chunk, n_iter - done)
                if k not in cache:
                    cache[k] = self.capture_steps(k, trace=trace, trace_capacity=chunk, accept_trace=acc_tr)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                # the trace record of iteration it goes to slot (it - 1) % chunk: a
                # run resumed at an iteration that is not a multiple of chunk starts
                # mid-ring
                r0 = self.iteration % chunk
                e0.record()
                cache[k].replay()
                self.iteration += k
                e1.record()
                h0, h1 = (0 if done == 0 else off + done), off + done + k
                if r0 == 0:
                    H[off + done:h1].copy_(trace[:k])
                else:
                    H[off + done:h1].copy_(trace[(torch.arange(k) + r0) % chunk])
                A[done:done + k].copy_(acc_tr[:k])
                if gather is None:
                    ev = torch.cuda.Event()
                    ev.record()
                    cs.wait_event(ev)
                    with torch.cuda.stream(cs):
                        Hh[h0:h1].copy_(H[h0:h1], non_blocking=True)
                        Ah[done:done + k].copy_(A[done:done + k], non_blocking=True)
                if timings:
                    e1.synchronize()
                    t_steps += [e0.elapsed_time(e1) * 1e-3 / k] * k
                done += k
            # the last step's flags, as the eager path leaves them in runner.accept
            if self.kind != "centered":
                self.accept.copy_(acc_tr[k - 1][:, :self.accept.shape[1]])
            self.graph = None
            p.iteration_counter(False)
            n_iter = 0
            if gather is None:
                cs.synchronize()
                H, A = Hh, Ah
        for i in range(n_iter):
            t0 = time.perf_counter() if timings else 0.0
            self.step()
            H[i + (1 if with_start else 0)].copy_(self.dl)
            if self.kind != "centered":
                A[i].copy_(self.accept)
            if timings:
                torch.cuda.synchronize()
                t_steps.append(time.perf_counter() - t0)
        if gather is not None:
            H = gather(H, dim=1)
            if self.kind != "centered":
                A = gather(A, dim=1)
        Hn = H.cpu().numpy()
        hist = {s: Hn[:, :, k, :len(p.bins[s]) - 1] for k, s in enumerate(p.spectra)}
        acc = None
        if self.kind != "centered":
            An = A.cpu().numpy()
            acc, off = {}, 0
            for s in MH_ORDER[p.F]:
                n = (len(p.blocks[s]) - 1) * p.n_iter_metropolis
                acc[s] = An[:, :, off:off + n]
                off += n
        if timings:
            return hist, acc, np.array(t_steps)
        return hist, acc

    def skymap(self):
        """Current sky map [nchains, F, (L+1)^2] as the reference would hold it
        (for ASIS with lazy re-centring the re-centred map is materialised here)."""
        if self.s is None:
            return None
        s = self.s.clone()
        if self.kind == "asis" and not self.materialize_recentre and self.iteration > 0:
            # ASIS.py:203 quirk: s <- A(C_new) s; corrected: s <- A(C_new) A(C_tmp)^+ s
            quirk = bool(self.quirks & C.GS_QUIRK_ASIS_RECENTRE_CENTERED)
            self.plan.recentre(self.dl, s, None if quirk else self.dl_tmp)
        return s

