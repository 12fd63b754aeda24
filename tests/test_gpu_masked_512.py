"""GPU: HEAD's masked ASIS at BASELINE configs[3]'s resolution (VERDICT r05
missing #1): N_side 512, l_max 1024, EB, the reference's own ASIS instantiation
(main_polarization.py:123-126: all_sph=False, gibbs_cr=True, n_gibbs=20,
overrelaxation=True; loop ASIS.py:134-226) on the matrix-core table path with 4
chains.  The dense oracle SHT cannot run at this size, so -- as for configs[4]
(tests/test_gpu_baseline_configs.py) -- the step is checked through
size-independent properties:

* one aux-variable CR step of a 4-chain table-path context
  (CenteredGibbs.py:676-729): every chain's v | s draw recovered to the
  oracle's Philox normals (chain key = chain0 + b) on sampled pixels and
  N(0, 1) over all its pixels, and its s | v draw against the oracle's per-l
  EB block algebra (H.centered_params, kappa = mu / w) on sampled slots, given
  the step's own analysis of v + N^-1 d;
* one full masked ASIS iteration (over-relaxed aux CR, centred C_l draw,
  non-centring, the pixel-domain MH f2, re-centring) of the 4-chain batch:
  chain 2's D_l and every accept flag equal a one-chain run of global chain 2
  (the batch contract of the table path: each chain's arithmetic is its
  one-chain run's), and the drawn D_l are finite and positive.
"""
import math

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import harmonic as H  # noqa: E402
from oracle import masked as MK  # noqa: E402

pytestmark = pytest.mark.gpu
SEED = 20261018
N, L = 512, 1024


@pytest.fixture(scope="module")
def data():
    from gibbssampler_amd.data import band_mask
    from gibbssampler_amd.problem import fiducial_dl, gauss_beam
    npix = 12 * N * N
    g = torch.Generator(device="cuda").manual_seed(11)
    mask = torch.from_numpy(band_mask(N)).cuda()
    maps = torch.randn((2, npix), generator=g, device="cuda", dtype=torch.float64) * 0.2 * mask
    return dict(Q=maps[0].cpu().numpy(), U=maps[1].cpu().numpy(), mask=mask.cpu().numpy(),
                bl=gauss_beam(math.radians(0.5), L), dl=fiducial_dl(L, 2))


def test_aux_step_512_tables_4chains(data):
    from gibbssampler_amd import _capi
    from gibbssampler_amd.masked import MaskedCR
    from gibbssampler_amd.sht import HealpixSHT
    F, B, chain0, it = 2, 4, 5, 3
    npix, NR = 12 * N * N, (L + 1) ** 2
    cr = MaskedCR({"Q": data["Q"], "U": data["U"]}, 40.0 ** 2, 0.2 ** 2, data["bl"], L, N, mask=data["mask"],
                  nfields=F, gibbs_cr=True, n_gibbs=1, rng="native", seed=SEED, chain=chain0, nchains=B,
                  sht_mode="mfma")
    assert cr.sht_tables
    dl = np.stack([data["dl"]["EE"], data["dl"]["BB"]])
    dl_t = torch.from_numpy(np.array(np.broadcast_to(dl, (B,) + dl.shape))).cuda().contiguous()
    g = torch.Generator(device="cuda").manual_seed(3)
    s0 = torch.randn((B, F, NR), generator=g, device="cuda", dtype=torch.float64) * 1e-2
    s = s0.clone()
    cr.step(_capi.GS_MCR_AUX, dl_t, s, iteration=it)
    torch.cuda.synchronize()
    v = cr.v.reshape(B, F, npix)
    sht = HealpixSHT(N, L)
    bl_t = torch.from_numpy(data["bl"]).cuda()
    ell = torch.from_numpy(H.slot_ell(L)).cuda()
    mask = torch.from_numpy(data["mask"]).cuda()
    inv = mask[None] / (0.2 ** 2)
    mu = torch.from_numpy(np.asarray(cr.mu)[1:3]).cuda()
    gam = mu[:, None] - inv
    maps = torch.from_numpy(np.stack([data["Q"], data["U"]])).cuda()
    mm_model = H.Model(L, N, F, data["bl"], [1.0 / float(cr.mu[k]) for k in (1, 2)],
                       {sp: np.arange(L + 2) for sp in H.SPECTRA[2]})
    M, Lc = H.centered_params(mm_model, dl)
    ls, _ = H.complex_ell_m(L)
    rng = np.random.default_rng(1)
    pix = np.concatenate([np.arange(64), rng.integers(0, npix, 3000), [npix - 1]]).astype(np.uint64)
    i_c = np.concatenate([np.arange(L + 1), rng.integers(L + 1, (L + 1) * (L + 2) // 2, 4000)]).astype(np.uint64)
    ii = i_c.astype(np.int64)
    for b in range(B):
        k0, k1 = H.chain_key(SEED, chain0 + b)
        # v | s: v = gamma A b s + sqrt(gamma) z (CenteredGibbs.py:693-700), rows Q, U
        Abs = sht.alm2map(s0[b] * bl_t[ell][None], ncomp=F)
        zhat = (v[b] - gam * Abs) / gam.sqrt()
        n = zhat.numel()
        mean, var = float(zhat.mean()), float(zhat.var())
        assert abs(mean) < 6.0 / math.sqrt(n) and abs(var - 1.0) < 6.0 * math.sqrt(2.0 / n), (b, mean, var)
        for k, row in enumerate((1, 2)):
            w = H.philox4x32_10(pix, row, MK.TAG_AUX_V | (0 << 8), it, k0, k1)
            zo = H.box_muller(*w)[0]
            np.testing.assert_allclose(zhat[k, pix.astype(np.int64)].cpu().numpy(), zo, rtol=0, atol=1e-6,
                                       err_msg=f"chain {b} row {row}")
        del Abs, zhat
        # s | v on sampled slots: s = M (map2alm(v + N^-1 d) / mu) + Lc z
        r_real = sht.map2alm(v[b] + inv * maps, ncomp=F).cpu().numpy()
        got = s[b].cpu().numpy()
        w = H.philox4x32_10(i_c[None, :], np.arange(F, dtype=np.uint64)[:, None], H.TAG_CR | (MK.SUB_S << 8), it,
                            k0, k1)
        z0, z1 = H.box_muller(*w)
        for part, zz in ((0, z0), (1, z1)):
            sel = ii if part == 0 else ii[ii > L]
            if part == 1:
                zz = zz[:, ii > L]
            slot = np.where(sel <= L, sel, 2 * sel - (L + 1) + part)
            d_eff = r_real[:, slot] / np.asarray(cr.mu)[1:3, None]
            lv = ls[sel]
            want = np.einsum("sfg,gs->fs", M[lv], d_eff) + np.einsum("sfg,gs->fs", Lc[lv], zz)
            np.testing.assert_allclose(got[:, slot], want, rtol=1e-9, atol=1e-12 * np.abs(want).max(),
                                       err_msg=f"chain {b} s | v part {part}")


def test_masked_asis_512_batch_equals_single(data):
    from gibbssampler_amd import gibbs as G
    from gibbssampler_amd.problem import bin_spectrum, default_bins, default_blocks, proposal_variances
    npix = 12 * N * N
    bins = default_bins(L, 2)
    blocks = default_blocks(L, bins)
    pv = proposal_variances(L, N, bins, data["bl"], 0.2 ** 2, 40.0 ** 2, fsky=float(np.mean(data["mask"])))
    init = {s: bin_spectrum(data["dl"][s], bins[s]) for s in ("EE", "BB")}
    pix = {"Q": data["Q"], "U": data["U"]}

    def run(nch, chain0):
        smp = G.ASIS(pix, np.ones(npix) * 40.0 ** 2, np.ones(npix) * 0.2 ** 2, 0.5, N, L, npix, pv,
                     metropolis_blocks=blocks, n_iter=1, all_sph=False, gibbs_cr=True, n_gibbs=20,
                     overrelaxation=True, mask_path=data["mask"], polarization=True, bins=bins, rng="native",
                     seed=SEED, chain0=chain0, nchains=nch, sht_mode="mfma")
        out = smp.masked_runner.run(init, 1)
        torch.cuda.synchronize()
        return out[0], out[1]

    h4, a4 = run(4, 0)
    h1, a1 = run(1, 2)
    for sp in ("EE", "BB"):
        assert np.all(np.isfinite(h4[sp])) and np.all(h4[sp][-1][:, 2:] > 0), sp
        np.testing.assert_array_equal(h4[sp][:, 2], h1[sp], err_msg=sp)
        np.testing.assert_array_equal(a4[sp][:, 2], a1[sp], err_msg=sp)
    assert sum(int(a4[sp].sum()) for sp in ("EE", "BB")) > 0
