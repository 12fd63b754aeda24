"""GPU: the constant-weight ring forms (k_ring_classes, gs_sht_register_weights).

A masked context registers its N^-1 once.  On ring pairs whose weights are one
number per ring (isotropic noise -- the reference's noise_temp / noise_pol are
np.ones(Npix) * var, main_polarization.py:105-107 -- on rings the mask leaves
whole) two ring-stage shortcuts apply, both exact in arithmetic and different
from the pixel route only in rounding:
  * the PCG operator's fused ring stage (k_sht_apply_ring_mc): inverse DFT,
    weight, forward DFT = n w per bin (CenteredGibbs.py:448-491's operator);
  * the f2 Gram pass (NonCenteredGibbs.py:333-355): block maps and the residual
    in Parseval coordinates on such rings, no ring DFT for the block maps.
Checked here with isotropic noise on the SURVEY band mask (every ring whole or
cut) and on a wavy galactic-like mask (rings crossing the edge stay on the
pixel route): against the oracle (the same tolerances as tests/test_gpu_masked.py),
against the pixel route (GS_SHT_CONST_RINGS=0) and batch == one chain bit for bit.
"""
import numpy as np
import pytest

from oracle import masked as MK

pytestmark = pytest.mark.gpu


def _close(got, want, rtol=1e-9):
    np.testing.assert_allclose(got, want, rtol=rtol, atol=1e-11 * np.abs(want).max())


def _problem(N, L, maskkind, seed=3):
    from gibbssampler_amd.data import band_mask, galactic_mask
    rng = np.random.default_rng(seed)
    npix = 12 * N * N
    mask = band_mask(N) if maskkind == "band" else galactic_mask(N)
    maps = rng.standard_normal((3, npix)) * np.array([[30.0], [0.3], [0.3]])
    ntemp, npol = np.full(npix, 40.0 ** 2), np.full(npix, 0.2 ** 2)      # isotropic noise
    ell = np.arange(L + 1)
    bl = np.exp(-0.5 * ell * (ell + 1) * (0.07 / np.sqrt(8 * np.log(2))) ** 2)
    dl = {"TT": np.where(ell >= 2, 1000.0, 0.0), "EE": np.where(ell >= 2, 10.0 * (np.maximum(ell, 1) / 100) ** 0.5, 0),
          "BB": np.where(ell >= 2, 0.01, 0.0)}
    dl["TE"] = 0.5 * np.sqrt(dl["TT"] * dl["EE"])
    s0 = rng.standard_normal((3, (L + 1) ** 2)) * np.array([[3.0], [0.05], [0.005]])
    return mask, maps, ntemp, npol, bl, dl, s0


def _cr(N, L, maskkind, F=2, **kw):
    from gibbssampler_amd.masked import MaskedCR
    mask, maps, ntemp, npol, bl, dl, s0 = _problem(N, L, maskkind)
    cr = MaskedCR({"T": maps[0], "Q": maps[1], "U": maps[2]}, ntemp, npol, bl, L, N, mask=mask, nfields=F, **kw)
    mm = MK.MaskedModel(L, N, F, bl, maps, np.stack([mask / ntemp, mask / npol, mask / npol]))
    return cr, mm, dl, s0


def _spec(F):
    return ("EE", "BB") if F == 2 else ("TT", "EE", "BB", "TE")


@pytest.mark.parametrize("maskkind", ["band", "galactic"])
@pytest.mark.parametrize("F", [2, 3])
def test_operator_vs_oracle_and_pixel_route(gsopt, maskkind, F):
    """Q x (the fused operator on tables, constant-ring shortcut) against the
    oracle's pcg_operator and against the pixel route of the same context."""
    import torch
    N, L = 16, 32
    cr, mm, dl, s0 = _cr(N, L, maskkind, F=F, gibbs_cr=False, ula=False, sht_mode="mfma", rng="native")
    rows = (1, 2) if F == 2 else (0, 1, 2)
    dlu = np.stack([dl[k] for k in _spec(F)])
    x = np.stack([s0[r] for r in rows]) * 10.0
    dl_t, x_t = torch.from_numpy(dlu).cuda(), torch.from_numpy(np.ascontiguousarray(x)).cuda()
    got = cr.pcg_apply(dl_t, x_t).cpu().numpy()
    want = MK.pcg_operator(mm, dlu, x)
    for k in range(F):
        _close(got[k], want[k], rtol=1e-10)
    gsopt.setenv("GS_SHT_CONST_RINGS", "0")
    pix = cr.pcg_apply(dl_t, x_t).cpu().numpy()
    np.testing.assert_allclose(got, pix, rtol=1e-12, atol=1e-14 * np.abs(pix).max())
    assert not np.array_equal(got, pix)            # the shortcut did run (rounding differs)


@pytest.mark.parametrize("maskkind", ["band", "galactic"])
def test_pcg_solve_vs_oracle(maskkind):
    import torch
    N, L = 16, 32
    cr, mm, dl, s0 = _cr(N, L, maskkind, gibbs_cr=False, ula=False, sht_mode="mfma", rng="native")
    rng = np.random.default_rng(3)
    rhs = rng.standard_normal((2, (L + 1) ** 2)) * 10
    rhs[:, mm.slot_ell < 2] = 0.0
    dlu = np.stack([dl["EE"], dl["BB"]])
    want, _ = MK.pcg_solve(mm, dlu, rhs, tol=1e-13)
    x = cr.pcg_solve(torch.from_numpy(dlu).cuda(), torch.from_numpy(rhs).cuda(), tol=1e-13).cpu().numpy()
    assert cr.pcg_residual <= 1e-13
    _close(x, want)


def _mh_parts(L):
    bins = {"EE": np.arange(L + 2), "BB": np.array([0, 2, 5, 9, 13, 17, 22, 27, L + 1])}
    blocks = {"EE": np.array([2, 10, L + 1]), "BB": np.array([2, 3, 4, 5, 6, 7, 8])}
    ell = np.arange(2, L + 1)
    pv = {"EE": (0.05 * 10.0 * (ell / 100.0) ** 0.5) ** 2, "BB": np.full(len(bins["BB"]) - 3, (0.2 * 0.01) ** 2)}
    return bins, blocks, pv


def _mh_model(mm, L, N, bl, bins, blocks, pv):
    from oracle import harmonic as H
    return H.Model(L, N, 2, bl, [1.0, 1.0], bins, blocks=blocks, proposal_variances=pv,
                   d_alm=np.zeros((2, (L + 1) ** 2)))


@pytest.mark.parametrize("sht_mode", ["recurrence", "mfma"])
@pytest.mark.parametrize("maskkind,group", [("band", None), ("galactic", None), ("galactic", "1")])
def test_pixel_mh_parseval_vs_oracle(gsopt, maskkind, group, sht_mode):
    """one f2 sweep (native streams) with the Parseval rows against the oracle's
    full-map likelihood per block, and equal to the pixel route's decisions;
    group "1": one block per Gram group (the residual carried between groups
    in the mixed coordinates)."""
    from gibbssampler_amd.masked import PixelMH
    if group is not None:
        gsopt.setenv("GS_F2_GROUP_BYTES", group)
    N, L = 16, 32
    cr, mm, dl, s0 = _cr(N, L, maskkind, gibbs_cr=False, ula=False, rng="native", seed=77, chain=3,
                         sht_mode=sht_mode)
    bins, blocks, pv = _mh_parts(L)
    mh = PixelMH(cr, bins, blocks, pv)
    snc = s0[1:] * 40.0
    init = {"EE": dl["EE"][:L + 1].copy(),
            "BB": np.array([np.mean(dl["BB"][bins["BB"][i]:bins["BB"][i + 1]]) for i in range(len(bins["BB"]) - 1)])}
    new, acc = mh.sample(snc, init, iteration=5)
    model = _mh_model(mm, L, N, cr.bl, bins, blocks, pv)
    want, wacc = MK.pixel_mh(mm, model, init, snc, seed=77, chain=3, iteration=5)
    _close(new["EE"], want["EE"])
    _close(new["BB"], want["BB"])
    assert acc == wacc
    n_acc = sum(int(np.sum(v)) for v in acc.values())
    assert 0 < n_acc < mh.K                          # both decision branches
    gsopt.setenv("GS_SHT_CONST_RINGS", "0")
    new0, acc0 = mh.sample(snc, init, iteration=5)
    assert acc0 == acc
    for sp in ("EE", "BB"):
        np.testing.assert_array_equal(new0[sp], new[sp])   # same decisions -> the same proposals kept


@pytest.mark.parametrize("maskkind", ["band", "galactic"])
def test_batch_equals_single_const_rings(maskkind):
    """chain b of a 4-chain context = a one-chain context of id chain0 + b, bit
    for bit, through the constant-ring operator (PCG) and the Parseval f2 sweep."""
    import torch
    from gibbssampler_amd.masked import PixelMH
    N, L, B, c0 = 16, 32, 4, 2
    kw = dict(gibbs_cr=False, ula=False, rng="native", seed=11, sht_mode="mfma", pcg_accuracy=1e-9)
    batch, mm, dl, s0 = _cr(N, L, maskkind, chain=c0, nchains=B, **kw)
    ones = [_cr(N, L, maskkind, chain=c0 + b, **kw)[0] for b in range(B)]
    dlu = np.stack([dl["EE"], dl["BB"]])
    dlb = torch.from_numpy(np.stack([dlu * (1.0 + 0.1 * b) for b in range(B)])).cuda()
    xb = batch.pcg_solve(dlb, batch.pcg_rhs(dlb, iteration=2))
    for b in range(B):
        d1 = dlb[b].contiguous()
        assert torch.equal(xb[b], ones[b].pcg_solve(d1, ones[b].pcg_rhs(d1, iteration=2))), f"pcg chain {b}"
    bins, blocks, pv = _mh_parts(L)
    mhb = PixelMH(batch, bins, blocks, pv)
    start = {"EE": dl["EE"][:L + 1].copy(),
             "BB": np.array([np.mean(dl["BB"][bins["BB"][i]:bins["BB"][i + 1]]) for i in range(len(bins["BB"]) - 1)])}
    inits = [{k: v * (1.0 + 0.05 * b) for k, v in start.items()} for b in range(B)]
    snc = torch.from_numpy(np.ascontiguousarray(np.stack([s0[1:] * (30.0 + b) for b in range(B)]))).cuda()
    out_b, fl_b = mhb.sweep_t(snc, mhb.plan.dl_tensor(inits), 5)
    out_b, fl_b = out_b.cpu().numpy(), fl_b.cpu().numpy().copy()
    for b in range(B):
        mh1 = PixelMH(ones[b], bins, blocks, pv)
        o1, f1 = mh1.sweep_t(snc[b].contiguous(), mh1.plan.dl_tensor(inits[b])[0], 5)
        np.testing.assert_array_equal(out_b[b], o1.cpu().numpy(), err_msg=f"mh chain {b}")
        np.testing.assert_array_equal(fl_b[b], f1.cpu().numpy(), err_msg=f"mh chain {b}")
