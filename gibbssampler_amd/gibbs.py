"""The reference's class surface (drop-in for main_polarization.py), backed by the HIP path.

Mirrors Gabriel-Ducrocq/GibbsSampler:
  GibbsSampler        GibbsSampler.py:8-192
  CenteredGibbs       CenteredGibbs.py:859-876
  NonCenteredGibbs    NonCenteredGibbs.py:449-582
  ASIS                ASIS.py:16-233
and the step samplers the drivers own (``constrained_sampler``,
``cls_sampler``; ``centered_cls_sampler`` / ``non_centered_cls_sampler``
for ASIS) with the same ``sample`` signatures and return conventions.

What the build covers (BASELINE.json north_star): the full-sky,
isotropic-noise harmonic path (``mask_path=None``; ``all_sph`` semantics) for
T-only, EB (the reference's polarization runs) and TEB.  The reference's
centered full-sky runs go through its PCG branch (CenteredGibbs.py:845-850,
qcinv); on the full sky with isotropic noise that system is diagonal and the
closed form (CenteredGibbs.py:317-353) is its exact solution, which is what
runs here.  Masked centered runs (``mask_path`` = mask array or .npy file)
use the device SHT and the PCG / auxiliary-variable / over-relaxation /
MALA samplers of gibbssampler_amd.masked (CenteredGibbs.py:448-850, the a12
flag ladder; the PCG is the init CR as at HEAD); masked NonCenteredGibbs and
ASIS score the MH blocks with the pixel-domain likelihood
(NonCenteredGibbs.py:333-355, gibbssampler_amd.masked.PixelMH).  ``mask_path``
is a HEALPix FITS file (any N_side, ud_graded), a .npy file or an array.
Masked-only keywords: ``n_gibbs``, ``alpha``, ``tau``, ``skymap_init`` (a
start map instead of the reference's PCG init CR).  Full-sky data may be
given as pixel maps (Q, U[, T]); they are analysed once with map2alm(iter=3).

Extra keyword arguments (all optional): ``nchains`` (batched chains on one
GPU), ``rng`` ("native" Philox or "replay" = numpy's global RNG in the
reference's draw order), ``seed`` (native streams), ``fields`` ("EB" or
"TEB" for polarization), ``chain0`` (global id of the first chain),
``reference_quirks`` (ASIS re-centring of the centered map, ASIS.py:203),
``distributed`` (one process per GPU under torchrun: this rank runs global
chains [rank * nchains, (rank + 1) * nchains) and ``run()`` returns every
rank's chains, all-gathered over RCCL -- the reference's SLURM array,
job-script.sh:6-8), ``dist_backend`` ("nccl" = RCCL, or "gloo"),
``keep_skymap`` (full-sky runs: keep each iteration's CR map on the device
for the ``skymap`` property; off by default -- the reference's ``run`` returns
D_l and accept histories only, and without the map store the CR sweep is ~20 %
faster).
"""
import os
import time

import numpy as np
import torch

from .problem import gauss_beam
from . import _capi as C

_SPECTRA = {1: ("TT",), 2: ("EE", "BB"), 3: ("TT", "EE", "BB", "TE")}


def _nfields(polarization, fields):
    if not polarization:
        return 1
    if fields is None or fields.upper() == "EB":
        return 2
    if fields.upper() == "TEB":
        return 3
    raise ValueError("fields must be 'EB' or 'TEB'")


def _scalar_noise(noise, what):
    a = np.atleast_1d(np.asarray(noise, dtype=np.float64))
    if not np.all(a == a.flat[0]):
        raise NotImplementedError(f"{what}: anisotropic pixel noise needs the pixel-domain (SHT) path")
    return float(a.flat[0])


def _harmonic_data(pix_map, nfields, lmax, nside):
    """Real-layout harmonic data d_alm per field.  Given as a_lm under
    'TT'/'EE'/'BB' (the all_sph form, main_polarization.py:43-45), or as pixel
    maps ('Q'/'U', plus 'T' or 'I' for TEB; an Npix array for TT), analysed
    once on the device with map2alm(iter=3) -- the non-all_sph data term of
    NonCenteredGibbs.py:155-159 / utils.adjoint_synthesis_hp, which the
    reference recomputes every iteration."""
    keys = {1: ("TT",), 2: ("EE", "BB"), 3: ("TT", "EE", "BB")}[nfields]
    npix = 12 * nside ** 2
    if nfields == 1 and not isinstance(pix_map, dict):
        arr = np.asarray(pix_map, dtype=np.float64)
        if arr.shape[-1] == (lmax + 1) ** 2:
            return {"TT": arr}
        if arr.shape[-1] != npix:
            raise ValueError("TT data must be a real-layout a_lm or an Npix map")
        return {"TT": _analyse([arr], nside, lmax)[0]}
    if all(k in pix_map for k in keys):
        return {k: np.asarray(pix_map[k], dtype=np.float64) for k in keys}
    if "Q" in pix_map and "U" in pix_map:
        if nfields == 2:
            a = _analyse([pix_map["Q"], pix_map["U"]], nside, lmax)
            return {"EE": a[0], "BB": a[1]}
        t = pix_map.get("T", pix_map.get("I"))
        if t is not None:
            a = _analyse([t, pix_map["Q"], pix_map["U"]], nside, lmax)
            return {"TT": a[0], "EE": a[1], "BB": a[2]}
    raise ValueError(f"pix_map needs harmonic data {keys} or pixel maps (Q, U[, T])")


def _analyse(maps, nside, lmax):
    import torch
    from .sht import HealpixSHT
    m = torch.as_tensor(np.ascontiguousarray(np.stack([np.asarray(x, dtype=np.float64) for x in maps])),
                        device="cuda")
    sht = HealpixSHT(nside, lmax)
    a = sht.map2alm(m if len(maps) > 1 else m[0], iter=3, ncomp=len(maps))
    return a.reshape(len(maps), -1).cpu().numpy()


def _load_mask(mask_path, nside):
    """The mask of CenteredGibbs.py:266-271 (hp.ud_grade(hp.read_map(path), nside)):
    a HEALPix FITS map (io.read_map, RING or NESTED), a .npy file or an array,
    brought to the run's N_side with io.ud_grade."""
    from . import io as gio
    if isinstance(mask_path, np.ndarray):
        m = np.asarray(mask_path, dtype=np.float64)
    elif isinstance(mask_path, str) and mask_path.endswith(".npy"):
        m = np.load(mask_path, allow_pickle=False).astype(np.float64)
    elif isinstance(mask_path, str):
        m = gio.read_map(mask_path, 0)
    else:
        raise TypeError("mask_path: a FITS / .npy path or an array")
    if m.ndim != 1:
        raise ValueError("mask must be one HEALPix map")
    if m.shape != (12 * nside ** 2,):
        m = gio.ud_grade(m, nside)
    return m


def _default_bins(lmax, nfields):
    return {s: np.arange(0, lmax + 2) for s in _SPECTRA[nfields]}


def _default_blocks(bins):
    """MHClsSampler default (ClsSampler.py:66-67): one block per bin from bin 2."""
    return {s: np.arange(2, len(b)) for s, b in bins.items()}


class GibbsSampler:
    """GibbsSampler.py:8-192."""

    _kind = None

    def __init__(self, pix_map, noise, beam_fwhm_deg, nside, lmax, polarization=False, bins=None, n_iter=10000,
                 gibbs_cr=False, rj_step=False, ula=False, *, nchains=1, rng="native", seed=0, fields=None,
                 chain0=0, reference_quirks=True, noise_pol=None, proposal_variances=None,
                 metropolis_blocks=None, n_iter_metropolis=1, mask_path=None, distributed=False,
                 dist_backend=None, keep_skymap=False, sht_mode="auto"):
        self.shard = None
        # masked / pixel-TT runs: the Legendre stage of their transforms ("auto":
        # matrix-core tables from 4 chains on small maps, else the recurrence;
        # "recurrence"; "mfma").  Chain b of a batch equals a one-chain run of
        # the same chain id bit for bit only for the same resolved mode.
        self.sht_mode = sht_mode
        self.keep_skymap = bool(keep_skymap)
        if distributed:
            # one process per GPU under torchrun: this rank runs global chains
            # [rank * nchains, (rank + 1) * nchains); run() returns every rank's
            # chains (histories all-gathered over RCCL) -- the role of the
            # reference's SLURM array (job-script.sh:6-8)
            import torch
            from .distributed import ShardContext
            backend = dist_backend or ("nccl" if torch.cuda.is_available() else "gloo")
            self.shard = ShardContext(nchains, backend=backend)
            if backend == "nccl":
                torch.cuda.set_device(self.shard.local)
            chain0 = self.shard.chain0
        self.mask = None
        if mask_path is not None:
            self.mask = _load_mask(mask_path, nside)
        self.noise = noise
        self.beam = beam_fwhm_deg
        self.nside = nside
        self.lmax = lmax
        self.polarization = polarization
        self.Npix = 12 * nside ** 2
        self.n_iter = n_iter
        self.gibbs_cr = gibbs_cr
        self.rj_step = rj_step
        self.ula = True                      # GibbsSampler.py:41 (hard-coded)
        self.nfields = _nfields(polarization, fields)
        self.spectra = _SPECTRA[self.nfields]
        self.pix_map = pix_map
        self.bl_gauss = gauss_beam((np.pi / 180) * beam_fwhm_deg, lmax)
        self.bl_map = self.compute_bl_map(beam_fwhm_deg)
        if bins is None:
            self.bins = _default_bins(lmax, self.nfields)
        elif isinstance(bins, dict):
            self.bins = {s: np.asarray(bins[s]) for s in self.spectra}
        else:
            self.bins = {self.spectra[0]: np.asarray(bins)}
        self.dls_to_cls_array = np.array([2 * np.pi / (l * (l + 1)) if l != 0 else 0 for l in range(lmax + 1)])
        self.noise_pol = noise_pol
        # TT from a pixel map keeps per-pixel noise (the f4 pixel path); the harmonic
        # path needs isotropic noise and checks it when it is built
        tt_pixel_map = self.nfields == 1 and not isinstance(pix_map, dict) and \
            np.asarray(pix_map).shape[-1] == 12 * nside ** 2
        if self.mask is not None or tt_pixel_map:
            nt = float(np.atleast_1d(noise)[0])
        else:
            nt = _scalar_noise(noise, "noise")
        if self.mask is not None:
            npol = float(np.atleast_1d(noise_pol if noise_pol is not None else noise)[0])
            self.noise_var = np.array([npol, npol] if self.nfields == 2 else [nt, npol, npol])
        elif self.nfields == 1:
            noise_var = [nt]
        else:
            npol = _scalar_noise(noise_pol if noise_pol is not None else noise, "noise_pol")
            noise_var = [npol, npol] if self.nfields == 2 else [nt, npol, npol]
        if self.mask is None:
            self.noise_var = np.array(noise_var)
        self.nchains = int(nchains)
        self.rng = rng
        self.seed = seed
        self.chain0 = chain0
        self.reference_quirks = reference_quirks
        self.proposal_variances = proposal_variances
        self.metropolis_blocks = metropolis_blocks
        self.n_iter_metropolis = n_iter_metropolis
        self._runner = None
        self._tt = None

    # -- f4: temperature from pixel data (reference semantics, gibbssampler_amd.tt) -----------
    def _tt_pixel_path(self, all_sph):
        """TT runs on the pixel map itself (CenteredGibbs.py:103-236, NonCenteredGibbs.py:17-249)
        unless the caller asks for the all_sph / harmonic form or gives a_lm."""
        if self.nfields != 1 or all_sph:
            return False
        if self.mask is not None:
            return True
        return not isinstance(self.pix_map, dict) and np.asarray(self.pix_map).shape[-1] == self.Npix

    def _tt_model(self, with_mh):
        from .tt import TTModel
        if self._tt is None:
            # nchains > 1: one batch (batched SHTs), histories with a chain axis
            pm = self.pix_map["TT"] if isinstance(self.pix_map, dict) else self.pix_map
            pv = blocks = None
            if with_mh:
                pv = self.proposal_variances
                pv = pv["TT"] if isinstance(pv, dict) else pv
                blocks = self.metropolis_blocks
                blocks = blocks["TT"] if isinstance(blocks, dict) else blocks
            self._tt = TTModel(pm, self.noise, self.bl_gauss, self.lmax, self.nside, self.bins["TT"], mask=self.mask,
                               blocks=blocks, proposal_variances=pv, n_iter_metropolis=self.n_iter_metropolis,
                               rng=self.rng, seed=self.seed, chain=self.chain0, nchains=self.nchains,
                               sht_mode=self.sht_mode)
        return self._tt

    # -- helpers of the reference base class --------------------------------------------
    def dls_to_cls(self, dls_):
        """GibbsSampler.py:56-62."""
        return dls_[:] * self.dls_to_cls_array

    def compute_bl_map(self, beam_fwhm_deg):
        """GibbsSampler.py:64-74: b_l expanded to the real a_lm layout."""
        bl = gauss_beam((np.pi / 180) * beam_fwhm_deg, self.lmax)
        return np.concatenate([bl, np.array([cl for m in range(1, self.lmax + 1) for cl in bl[m:] for _ in range(2)])])

    # -- the device runner ------------------------------------------------------------------
    def _make_runner(self):
        from .samplers import BatchedRunner
        if self._runner is None:
            d = _harmonic_data(self.pix_map, self.nfields, self.lmax, self.nside)
            blocks = None
            pv = None
            if self._kind in ("noncentered", "asis"):
                blocks = self.metropolis_blocks if self.metropolis_blocks is not None else _default_blocks(self.bins)
                if isinstance(blocks, dict):
                    blocks = {s: np.asarray(blocks[s]) for s in self.spectra}
                else:
                    blocks = {self.spectra[0]: np.asarray(blocks)}
                pv = self.proposal_variances
                if not isinstance(pv, dict):
                    pv = {self.spectra[0]: np.asarray(pv)}
            self._runner = BatchedRunner(kind=self._kind, lmax=self.lmax, nside=self.nside, nfields=self.nfields,
                                         nchains=self.nchains, bl=self.bl_gauss, noise_var=self.noise_var,
                                         bins=self.bins, d_alm=d, blocks=blocks, proposal_variances=pv,
                                         rng=self.rng, seed=self.seed, chain0=self.chain0,
                                         quirks=C.GS_QUIRK_ASIS_RECENTRE_CENTERED if self.reference_quirks else 0,
                                         n_iter_metropolis=self.n_iter_metropolis,
                                         store_skymap=self.keep_skymap)
        return self._runner

    def _masked_cr(self, noise_temp, noise_pol, gibbs_cr=False, n_gibbs=1, alpha=-0.995, overrelaxation=False,
                   ula=False, tau=0.02, rj=False):
        from .masked import MaskedCR
        if not self.polarization:
            raise NotImplementedError("masked temperature-only runs: the reference's TT masked path is broken "
                                      "at HEAD (SURVEY.md Appendix B.7); use fields='TEB'")
        # nchains > 1: the chains run as one batch (batched SHTs, per-chain streams
        # keyed by the global chain id chain0 + b); histories gain a chain axis
        return MaskedCR(self.pix_map, noise_temp, noise_pol, self.bl_gauss, self.lmax, self.nside, mask=self.mask,
                        nfields=self.nfields, gibbs_cr=gibbs_cr, n_gibbs=n_gibbs, alpha=alpha,
                        overrelaxation=overrelaxation, ula=ula, tau=tau, rng=self.rng, seed=self.seed,
                        chain=self.chain0, rj=rj, nchains=self.nchains, sht_mode=self.sht_mode)

    def _masked_mh_runner(self, kind, cr, cr_kind_):
        from .masked import MaskedMHRunner
        if self.nfields != 2:
            raise NotImplementedError("masked non-centred sampling is the reference's EB model "
                                      "(PolarizationNonCenteredClsSampler, NonCenteredGibbs.py:255-445)")
        blocks = self.metropolis_blocks if self.metropolis_blocks is not None else _default_blocks(self.bins)
        return MaskedMHRunner(kind, cr, self.bins, {s: np.asarray(blocks[s]) for s in self.spectra},
                              self.proposal_variances, self.n_iter_metropolis, cr_kind_=cr_kind_,
                              quirk=self.reference_quirks)

    def _squeeze(self, a):
        return a[:, 0] if a.shape[1] == 1 else a

    def _run_common(self, dls_init):
        runner = self._make_runner()
        resume, self._resume_state = getattr(self, "_resume_state", None), None
        init = dls_init if isinstance(dls_init, dict) or resume is not None else {self.spectra[0]: dls_init}
        h, acc, t = runner.run(init, self.n_iter, timings=True,
                               gather=self.shard.gather if self.shard is not None else None, resume=resume)
        h = {s: self._squeeze(v) for s, v in h.items()}
        if acc is not None:
            acc = {s: self._squeeze(v) for s, v in acc.items()}
        return h, acc, t

    def run(self, dls_init, resume=None):
        """GibbsSampler.py:183-192.  resume: a checkpoint() state (or the path of
        a save_checkpoint file) to continue from instead of dls_init -- full-sky
        (all_sph) runs; the histories then start at the checkpoint's D_l."""
        if resume is not None:
            if self.mask is not None or getattr(self, "tt_pixel", False):
                raise NotImplementedError("resume: full-sky (all_sph) runs only")
            self._resume_state = self.load_checkpoint(resume) if isinstance(resume, (str, os.PathLike)) else resume
        return self.run_polarization(dls_init) if self.polarization else self.run_temperature(dls_init)

    # -- checkpoint / resume ---------------------------------------------
    def checkpoint(self):
        """State of the chains after the last run (samplers.BatchedRunner.state_dict)."""
        if self._runner is None:
            raise RuntimeError("checkpoint: nothing has run yet")
        return self._runner.state_dict()

    def save_checkpoint(self, path):
        torch.save(self.checkpoint(), path)

    @staticmethod
    def load_checkpoint(path):
        return torch.load(path, weights_only=True)

    def run_polarization(self, dls_init):
        raise NotImplementedError

    def run_temperature(self, dls_init):
        raise NotImplementedError

    @property
    def skymap(self):
        """Current batched sky map [nchains, F, (L+1)^2] (device tensor); None
        unless the sampler was built with keep_skymap=True."""
        return None if self._runner is None or self._runner.s is None else self._runner.skymap()


class CenteredGibbs(GibbsSampler):
    """CenteredGibbs.py:859-876 (full-sky closed-form CR + inverse-Gamma/Wishart C_l draw)."""

    _kind = "centered"

    def __init__(self, pix_map, noise_temp, noise_pol, beam, nside, lmax, Npix, mask_path=None,
                 polarization=False, bins=None, n_iter=100000, rj_step=False, all_sph=False, gibbs_cr=False,
                 overrelaxation=False, ula=False, **kw):
        # rj_step with a mask: HEAD's ladder never reaches sample_mask_rj (its
        # branch is "and False", CenteredGibbs.py:837), so the run is the PCG
        # CR, as at HEAD; rj_active=True turns the RJPO branch back on.
        # constrained_sampler.sample_mask_rj is callable either way.
        rj_active = bool(kw.pop("rj_active", False))
        self.n_gibbs = int(kw.pop("n_gibbs", 1))
        self.alpha = float(kw.pop("alpha", -0.995))
        self.tau = float(kw.pop("tau", 0.02))
        self.skymap_init = kw.pop("skymap_init", None)
        super().__init__(pix_map, noise_temp, beam, nside, lmax, polarization=polarization, bins=bins,
                         n_iter=n_iter, gibbs_cr=gibbs_cr, rj_step=rj_step, mask_path=mask_path,
                         noise_pol=noise_pol, **kw)
        self.all_sph = all_sph
        self.overrelaxation = overrelaxation
        self.cr_ula = ula
        self.tt_pixel = self._tt_pixel_path(all_sph)
        if self.tt_pixel:
            from .tt import TTCenteredConstrainedRealization, TTCenteredClsSampler
            m = self._tt_model(False)
            self.constrained_sampler = TTCenteredConstrainedRealization(m)
            self.cls_sampler = TTCenteredClsSampler(m)
            return
        if self.mask is not None:
            self.constrained_sampler = self._masked_cr(noise_temp, noise_pol, gibbs_cr=gibbs_cr, n_gibbs=self.n_gibbs,
                                                       alpha=self.alpha, overrelaxation=overrelaxation, ula=ula,
                                                       tau=self.tau, rj=rj_step and rj_active)
        else:
            self.constrained_sampler = CenteredConstrainedRealization(self)
        self.cls_sampler = CenteredClsSampler(self)

    def _run_masked(self, dls_init):
        from .masked import MaskedRunner
        runner = MaskedRunner(self.constrained_sampler, self.bins)
        F = self.nfields
        s0 = self.skymap_init
        if isinstance(s0, dict):
            s0 = np.stack([np.asarray(s0[k]) for k in (("EE", "BB") if F == 2 else ("TT", "EE", "BB"))])
        init = dls_init if isinstance(dls_init, dict) else {self.spectra[0]: dls_init}
        return runner.run(init, self.n_iter, s0)

    def run_polarization(self, dls_init):
        """GibbsSampler.run_polarization (GibbsSampler.py:118-180): returns
        (h_dls, h_accept_cr, h_duration_cr, h_duration_cls_sampling)."""
        if self.mask is not None:
            return self._run_masked(dls_init)
        h, _, t = self._run_common(dls_init)
        n = len(t)
        return h, np.ones(n, dtype=int), np.asarray(t), np.zeros(n)

    def run_temperature(self, dls_init):
        """GibbsSampler.run_temperature (GibbsSampler.py:76-116)."""
        if self.tt_pixel:
            return self._tt.run_centered(dls_init, self.n_iter)
        h, _, t = self._run_common(dls_init)
        return h["TT"], np.ones(len(t), dtype=int), list(t)


class NonCenteredGibbs(GibbsSampler):
    """NonCenteredGibbs.py:449-582 (all_sph: per-l block MH)."""

    _kind = "noncentered"

    def __init__(self, pix_map, noise_I, noise_Q, beam, nside, lmax, Npix, proposal_variances,
                 metropolis_blocks=None, polarization=False, bins=None, n_iter=10000, n_iter_metropolis=1,
                 mask_path=None, all_sph=False, **kw):
        super().__init__(pix_map, noise_I, beam, nside, lmax, polarization=polarization, bins=bins, n_iter=n_iter,
                         mask_path=mask_path, noise_pol=noise_Q, proposal_variances=proposal_variances,
                         metropolis_blocks=metropolis_blocks, n_iter_metropolis=n_iter_metropolis, **kw)
        self.all_sph = all_sph
        self.tt_pixel = self._tt_pixel_path(all_sph)
        if self.tt_pixel:
            from .tt import TTNonCenteredConstrainedRealization, TTNonCenteredClsSampler
            m = self._tt_model(True)
            self.constrained_sampler = TTNonCenteredConstrainedRealization(m)
            self.cls_sampler = TTNonCenteredClsSampler(m)
            return
        self.constrained_sampler = NonCenteredConstrainedRealization(self)
        self.cls_sampler = NonCenteredClsSampler(self)
        if self.mask is not None:
            # NonCenteredGibbs.py:104-131,178-196: PCG in the centred parametrisation, then C^-1/2
            from .masked import KIND_PCG
            self.masked_cr = self._masked_cr(noise_I, noise_Q)
            self.masked_runner = self._masked_mh_runner("noncentered", self.masked_cr, KIND_PCG)
            self.cls_sampler = self.masked_runner.mh

    def run_polarization(self, dls_init):
        """NonCenteredGibbs.py:529-571: (h_dls, total_accept, h_duration_cr, h_duration_cls)."""
        if self.mask is not None:
            h, acc = self.masked_runner.run(dls_init, self.n_iter)[:2]
            return h, acc, np.array([]), np.array([])
        h, acc, t = self._run_common(dls_init)
        return h, acc, np.array([]), np.array([])

    def run_temperature(self, dls_init):
        """NonCenteredGibbs.py:488-527: (h_dl, total_accept, h_time_seconds)."""
        if self.tt_pixel:
            return self._tt.run_noncentered(dls_init, self.n_iter)
        h, acc, t = self._run_common(dls_init)
        return h["TT"][1:], acc["TT"], np.asarray(t)


class ASIS(GibbsSampler):
    """ASIS.py:16-233 (interweaving: centered CR + C_l draw, non-centering, NC MH, re-centring)."""

    _kind = "asis"

    def __init__(self, pix_map, noise, noise_Q, beam, nside, lmax, Npix, proposal_variances, metropolis_blocks=None,
                 polarization=False, bins=None, n_iter=10000, n_iter_metropolis=1, mask_path=None, gibbs_cr=False,
                 rj_step=False, all_sph=False, n_gibbs=20, overrelaxation=False, **kw):
        super().__init__(pix_map, noise, beam, nside, lmax, polarization=polarization, bins=bins, n_iter=n_iter,
                         gibbs_cr=gibbs_cr, rj_step=rj_step, mask_path=mask_path, noise_pol=noise_Q,
                         proposal_variances=proposal_variances, metropolis_blocks=metropolis_blocks,
                         n_iter_metropolis=n_iter_metropolis, **kw)
        self.all_sph = all_sph
        self.n_gibbs = n_gibbs
        self.overrelaxation = overrelaxation
        self.tt_pixel = self._tt_pixel_path(all_sph)
        if self.tt_pixel:
            from .tt import TTCenteredConstrainedRealization, TTCenteredClsSampler, TTNonCenteredClsSampler
            m = self._tt_model(True)
            self.constrained_sampler = TTCenteredConstrainedRealization(m)
            self.centered_cls_sampler = TTCenteredClsSampler(m)
            self.non_centered_cls_sampler = TTNonCenteredClsSampler(m)
            return
        self.constrained_sampler = CenteredConstrainedRealization(self)
        self.constrained_sampler.n_gibbs = n_gibbs
        self.centered_cls_sampler = CenteredClsSampler(self)
        self.non_centered_cls_sampler = NonCenteredClsSampler(self)
        if self.mask is not None:
            # ASIS.py:55-66: PolarizedCenteredConstrainedRealization(gibbs_cr, n_gibbs, overrelaxation) with its
            # default ula=True (CenteredGibbs.py:243-244); PCG unless gibbs_cr / rj_step (ASIS.py:153-170)
            from .masked import KIND_PCG, cr_kind
            self.masked_cr = self._masked_cr(noise, noise_Q, gibbs_cr=gibbs_cr, n_gibbs=n_gibbs,
                                             overrelaxation=overrelaxation, ula=True)
            kind = cr_kind(gibbs_cr, overrelaxation, True) if (gibbs_cr or rj_step) else KIND_PCG
            self.masked_runner = self._masked_mh_runner("asis", self.masked_cr, kind)
            self.constrained_sampler = self.masked_cr
            self.non_centered_cls_sampler = self.masked_runner.mh

    def run_polarization(self, dls_init):
        """ASIS.py:134-226: (h_dls, total_accept, accept_cr|None, h_iteration_duration,
        h_duration_cr, h_duration_cls_sampling, h_duration_cls_nc_sampling)."""
        if self.mask is not None:
            h, acc, acc_cr, t_it, t_cr, t_cls, t_nc = self.masked_runner.run(dls_init, self.n_iter)
            return h, acc, (acc_cr if self.rj_step else None), t_it, t_cr, t_cls, t_nc
        h, acc, t = self._run_common(dls_init)
        z = np.zeros(len(t))
        return h, acc, None, np.asarray(t), z, z, z

    def run_temperature(self, dls_init):
        """ASIS.py:69-131: (h_dls, h_accept, h_accept_cr, h_time_seconds)."""
        if self.tt_pixel:
            return self._tt.run_asis(dls_init, self.n_iter, gibbs_cr=self.gibbs_cr)
        h, acc, t = self._run_common(dls_init)
        return h["TT"], acc["TT"], np.ones(len(t), dtype=int), np.asarray(t)


# ---------------------------------------------------------------------------------------
# single-step samplers (the objects the drivers own) -- numpy in / numpy out, one chain
# ---------------------------------------------------------------------------------------
class _StepBase:
    def __init__(self, owner):
        self.owner = owner
        self.lmax = owner.lmax
        self.nside = owner.nside
        self.Npix = owner.Npix
        self.bl_map = owner.bl_map
        self.bl_gauss = owner.bl_gauss
        self.pix_map = owner.pix_map
        self.mask_path = None
        self.pcg_accuracy = 1.0e-5          # CenteredGibbs.py:280 (kept for the result dict)
        self.gibbs_cr = owner.gibbs_cr
        self.n_gibbs = 1
        self._plan = None
        self._d = None

    def _unbinned_plan(self):
        """A 1-chain plan with unbinned spectra (the CR steps take unbinned D_l)."""
        from .engine import GibbsPlan
        if self._plan is None:
            o = self.owner
            bins = {s: np.arange(0, o.lmax + 2) for s in o.spectra}
            self._plan = GibbsPlan(o.lmax, o.nside, o.nfields, 1, o.bl_gauss, o.noise_var, bins)
            self._d = self._plan.data_tensor(_harmonic_data(o.pix_map, o.nfields, o.lmax, o.nside))
        return self._plan

    def _binned_plan(self):
        return self.owner._make_runner().plan

    def _as_dict(self, x):
        return x if isinstance(x, dict) else {self.owner.spectra[0]: x}

    def _fields_dict(self, s):
        keys = {1: ("TT",), 2: ("EE", "BB"), 3: ("TT", "EE", "BB")}[self.owner.nfields]
        out = {k: s[i] for i, k in enumerate(keys)}
        return out if self.owner.nfields != 1 else out["TT"]

    def _draw(self, mode, all_dls):
        p = self._unbinned_plan()
        dl = p.dl_tensor(self._as_dict(all_dls))
        z = p.replay_cr_normals() if self.owner.rng == "replay" else None
        self._it = getattr(self, "_it", 0) + 1
        params = p.block_params(mode, dl)
        s, _ = p.cr_sweep(self._d, params, z=z, seed=self.owner.seed, iteration=0xFFFF0000 + self._it)
        return self._fields_dict(s.cpu().numpy()[0])


class CenteredConstrainedRealization(_StepBase):
    """PolarizedCenteredConstrainedRealization.sample (CenteredGibbs.py:317-353, 828-850)
    / CenteredConstrainedRealization (CenteredGibbs.py:103-232), full sky."""

    def sample(self, all_dls, s_old=None, *args, **kw):
        return self._draw(C.GS_MODE_CENTERED, all_dls), 1

    sample_no_mask = sample


class NonCenteredConstrainedRealization(_StepBase):
    """PolarizedNonCenteredConstrainedRealization.sample_no_mask (NonCenteredGibbs.py:134-176);
    returns accept 0 like the reference (176)."""

    def sample(self, all_dls, *args, **kw):
        return self._draw(C.GS_MODE_NONCENTERED, all_dls), 0

    sample_no_mask = sample


class _StatsMixin:
    def _stats_of(self, alms):
        import torch
        p = self._binned_plan()
        o = self.owner
        keys = {1: ("TT",), 2: ("EE", "BB"), 3: ("TT", "EE", "BB")}[o.nfields]
        a = alms if isinstance(alms, dict) else {"TT": alms}
        s = torch.from_numpy(np.stack([np.asarray(a[k], dtype=np.float64) for k in keys])[None].copy()).to(p.device)
        st = p.zeros(1, p.nstat, p.L + 1)
        C.check(p.lib.gs_sweep_stats(p._h, C.ptr(self.owner._make_runner().d), C.ptr(s), C.ptr(st),
                                     C.stream_ptr()), "gs_sweep_stats")
        return st


class CenteredClsSampler(_StepBase, _StatsMixin):
    """PolarizedCenteredClsSampler.sample (CenteredGibbs.py:54-93) / CenteredClsSampler (24-48)."""

    def sample(self, alms):
        p = self._binned_plan()
        st = self._stats_of(alms)
        var = p.replay_invgamma() if self.owner.rng == "replay" else None
        self._it = getattr(self, "_it", 0) + 1
        out = p.dl_dicts(p.cls_draw(st, variates=var, seed=self.owner.seed, iteration=0xFFFE0000 + self._it))[0]
        return out if self.owner.nfields != 1 else out["TT"]


class NonCenteredClsSampler(_StepBase, _StatsMixin):
    """PolarizationNonCenteredClsSampler.sample (NonCenteredGibbs.py:401-445), all_sph."""

    def sample(self, s_nonCentered, binned_dls_old, *args):
        p = self._binned_plan()
        st = self._stats_of(s_nonCentered)
        dl = p.dl_tensor(self._as_dict(binned_dls_old))
        up = ua = None
        if self.owner.rng == "replay":
            up, ua = p.replay_mh_uniforms()
        self._it = getattr(self, "_it", 0) + 1
        acc = p.split_accept(p.nc_mh(st, dl, up, ua, seed=self.owner.seed, iteration=0xFFFD0000 + self._it))
        out = p.dl_dicts(dl)[0]
        acc = {s: list(v[0]) for s, v in acc.items()}
        if self.owner.nfields == 1:
            return out["TT"], acc["TT"]
        return out, acc
