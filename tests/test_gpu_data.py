"""GPU: the f3 data path -- synalm / synfast / generate_dataset on the device
against oracle/data.py (same numpy draws), FITS masks through the class
surface, and full-sky pixel-map input analysed once with map2alm(iter=3)."""
import numpy as np
import pytest

from oracle import data as OD
from oracle import harmonic as H
from oracle import sht as O

pytestmark = pytest.mark.gpu


def _cls(L, seed=0):
    rng = np.random.default_rng(seed)
    ell = np.arange(L + 1)
    tt = np.where(ell >= 2, 1000.0 / (ell + 1.0) ** 2, 0.0) * (1 + 0.1 * rng.random(L + 1))
    ee = np.where(ell >= 2, 10.0 / (ell + 1.0) ** 2, 0.0)
    bb = np.where(ell >= 2, 0.01 / (ell + 1.0) ** 2, 0.0)
    te = 0.5 * np.sqrt(tt * ee)
    return np.stack([tt, ee, bb, te])


def _close(a, b):
    np.testing.assert_allclose(a, b, rtol=1e-10, atol=1e-12 * np.abs(b).max())


@pytest.mark.parametrize("F", [1, 2, 3])
def test_synalm_vs_oracle(F):
    from gibbssampler_amd.data import synalm
    L = 24
    c = _cls(L)
    rows = {1: c[:1], 2: {"EE": c[1], "BB": c[2]}, 3: c}[F]
    nf = {1: 1, 2: 2, 3: 3}[F]
    z = np.random.default_rng(F).standard_normal((nf, (L + 1) ** 2))
    got = synalm(rows, L, np.radians(2.0), z=z).cpu().numpy()
    want = OD.synalm_real(list(c[:1]) if F == 1 else ([c[1], c[2]] if F == 2 else list(c)), L, np.radians(2.0), z)
    _close(got, want)


@pytest.mark.parametrize("variant", ["full", "masked", "tt"])
def test_generate_dataset_vs_oracle(variant):
    from gibbssampler_amd.data import generate_dataset
    N, L = 8, 16
    c = _cls(L, 1)
    th, _ = O.pixel_angles(N)
    mask = (np.abs(np.cos(th)) > 0.2).astype(float) if variant == "masked" else None
    pol = variant != "tt"
    np.random.seed(42)
    got = generate_dataset(c if pol else c[0], N, L, 3.0, 40.0 ** 2, 0.2 ** 2, polarization=pol, mask=mask)
    np.random.seed(42)
    want = OD.generate_dataset(c if pol else c[0], N, L, 3.0, 40.0 ** 2, 0.2 ** 2, polarization=pol, mask=mask)
    assert len(got) == len(want)
    if variant == "full":
        _close(got[0], want[0])
        for k in ("EE", "BB"):
            _close(got[1][k], want[1][k])
        for k in ("Q", "U"):
            _close(got[2][k], want[2][k])
    elif variant == "masked":
        _close(got[0], want[0])
        for k in ("Q", "U"):
            _close(got[1][k], want[1][k])
        assert np.all(got[1]["Q"][mask == 0] == 0)
    else:
        assert got[0] is None
        _close(got[2], want[2])
        _close(got[3], want[3])


def test_synfast_spectrum_statistics():
    """the sky drawn at N_side 32, L 64 has the input spectrum (chi^2 per l)."""
    from gibbssampler_amd.data import synalm
    L = 64
    c = _cls(L, 2)
    np.random.seed(3)
    a = synalm(c, L, 0.0).cpu().numpy()
    sl = H.slot_ell(L)
    for f, k in ((0, 0), (1, 1), (2, 2)):
        chat = np.bincount(sl, weights=a[f] ** 2) / (2 * np.arange(L + 1) + 1)
        ratio = chat[2:] / c[k][2:]
        assert abs(ratio.mean() - 1) < 0.05
    n = 2 * np.arange(L + 1) + 1
    chat_te = np.bincount(sl, weights=a[0] * a[1]) / n
    zte = (chat_te[2:] - c[3][2:]) / np.sqrt((c[0][2:] * c[1][2:] + c[3][2:] ** 2) / n[2:])
    assert abs(zte.mean()) < 4 / np.sqrt(len(zte)) and 0.5 < zte.std() < 1.5


def test_fits_mask_through_the_surface(tmp_path):
    """mask_path as a FITS file at a finer N_side = the ud_graded array."""
    from gibbssampler_amd import io as gio
    from gibbssampler_amd.gibbs import CenteredGibbs
    N, L = 8, 16
    th16, _ = O.pixel_angles(16)
    m16 = (np.abs(np.cos(th16)) > 0.2).astype(float)
    p = str(tmp_path / "mask.fits")
    gio.write_map(p, gio.reorder(m16, r2n=True), nest=True)
    m8 = gio.ud_grade(m16, 8)
    rng = np.random.default_rng(5)
    pix = {"Q": rng.standard_normal(12 * N * N), "U": rng.standard_normal(12 * N * N)}
    init = {"EE": np.r_[0, 0, np.full(L - 1, 2.0)], "BB": np.r_[0, 0, np.full(L - 1, 0.1)]}
    out = []
    for mp in (p, m8):
        cg = CenteredGibbs(pix, np.full(12 * N * N, 1600.0), np.full(12 * N * N, 0.04), 3.0, N, L, 12 * N * N,
                           mask_path=mp, polarization=True, n_iter=2, gibbs_cr=True, rng="native", seed=4,
                           n_gibbs=2)
        out.append(cg.run({k: v.copy() for k, v in init.items()})[0])
    for s in ("EE", "BB"):
        np.testing.assert_array_equal(out[0][s], out[1][s])


def test_fullsky_pixel_maps_input():
    """full-sky Q/U maps are analysed once (map2alm iter=3) -> same chain as
    the harmonic input computed by the oracle SHT."""
    from gibbssampler_amd.gibbs import NonCenteredGibbs
    N, L = 8, 16
    rng = np.random.default_rng(6)
    Q, U = rng.standard_normal((2, 12 * N * N))
    a = O.map2alm(np.stack([np.zeros(12 * N * N), Q, U]), N, L, iter=3)
    harm = {"EE": H.complex_to_real(a[1], L), "BB": H.complex_to_real(a[2], L)}
    pv = {"EE": np.full(L - 1, 1e-3), "BB": np.full(L - 1, 1e-4)}
    init = {"EE": np.r_[0, 0, np.full(L - 1, 2.0)], "BB": np.r_[0, 0, np.full(L - 1, 0.1)]}
    out = []
    for pm in ({"Q": Q, "U": U}, harm):
        nc = NonCenteredGibbs(pm, 1600.0, 0.04, 3.0, N, L, 12 * N * N, pv, polarization=True, n_iter=3,
                              rng="native", seed=8, all_sph=True)
        out.append(nc.run({k: v.copy() for k, v in init.items()})[0])
    for s in ("EE", "BB"):
        np.testing.assert_allclose(out[0][s], out[1][s], rtol=1e-9)


@pytest.mark.parametrize("pol", [False, True])
def test_adjoint_synthesis_hp_vs_oracle(pol):
    """utils.adjoint_synthesis_hp (utils.py:79-111): Npix/4pi complex_to_real(
    map2alm(map, iter=3)) times the beam diagonal, against the dense oracle."""
    from gibbssampler_amd import utils as U
    N, L = 8, 16
    rng = np.random.default_rng(5)
    maps = rng.standard_normal((3, O.npix(N))) if pol else rng.standard_normal(O.npix(N))
    bl = H.gauss_beam(np.radians(5.0), L)[H.slot_ell(L)]
    got = U.adjoint_synthesis_hp(maps, bl)
    want = O.map2alm(maps, N, L, iter=3)
    want = np.atleast_2d(want)
    resc = O.npix(N) / (4 * np.pi)
    ref = [H.complex_to_real(w, L) * resc * bl for w in want]
    if pol:
        assert len(got) == 3
        for g, r in zip(got, ref):
            np.testing.assert_allclose(g, r, rtol=0, atol=1e-10 * np.abs(r).max())
    else:
        np.testing.assert_allclose(got, ref[0], rtol=0, atol=1e-10 * np.abs(ref[0]).max())
