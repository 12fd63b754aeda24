"""CPU: the f3 data formats (gibbssampler_amd/io.py) -- HEALPix NESTED/RING
indexing, ud_grade, the FITS map reader/writer and the .npz run records.

No FITS file ships with the reference, so the FITS layer is pinned by the
FITS standard (hand-built header cards and big-endian tables here) and round
trips; nest2ring by the HEALPix hierarchy (children of NESTED pixel p are
4p..4p+3, adjacent on the sphere; face-local x points north-east) and the RING
pixel centres of oracle/sht.py."""
import os

import numpy as np
import pytest

from gibbssampler_amd import io as gio
from oracle import sht as O


def _unit(nside):
    th, ph = O.pixel_angles(nside)
    return np.stack([np.sin(th) * np.cos(ph), np.sin(th) * np.sin(ph), np.cos(th)], axis=1)


def test_nest2ring_bijection_and_base():
    np.testing.assert_array_equal(gio.nest2ring(1, np.arange(12)), np.arange(12))
    for nside in (2, 4, 8, 16):
        r = gio.nest2ring(nside, np.arange(12 * nside * nside))
        assert np.array_equal(np.sort(r), np.arange(12 * nside * nside))
        np.testing.assert_array_equal(gio.ring2nest(nside, r), np.arange(12 * nside * nside))


@pytest.mark.parametrize("nside", [1, 2, 4, 8, 16])
def test_nest_children_are_adjacent(nside):
    """the 4 children of each NESTED pixel lie within one parent pixel of it."""
    up = _unit(2 * nside)
    par = _unit(nside)
    n = 12 * nside * nside
    parent_ring = gio.nest2ring(nside, np.arange(n))
    child_ring = gio.nest2ring(2 * nside, np.arange(4 * n)).reshape(n, 4)
    dist = np.arccos(np.clip(np.einsum("ij,ikj->ik", par[parent_ring], up[child_ring]), -1, 1))
    res = np.sqrt(4 * np.pi / n)
    assert dist.max() < 0.9 * res
    # mean of the children directions points at the parent centre
    mean = up[child_ring].mean(axis=1)
    mean /= np.linalg.norm(mean, axis=1, keepdims=True)
    assert np.arccos(np.clip(np.sum(mean * par[parent_ring], axis=1), -1, 1)).max() < 0.35 * res


def test_nest_orientation_face0():
    """HEALPix convention: in face 0, child 3 (ix=iy=1) is north of child 0 and
    child 1 (ix=1) lies east (larger phi) of child 2 (iy=1)."""
    th, ph = O.pixel_angles(2)
    r = gio.nest2ring(2, np.arange(4))
    assert th[r[3]] < th[r[1]] < th[r[0]]
    assert th[r[1]] == pytest.approx(th[r[2]])
    assert ph[r[1]] > ph[r[2]]
    assert ph[r[0]] == pytest.approx(np.pi / 4) and np.cos(th[r[0]]) == pytest.approx(1 / 3)


def test_reorder_roundtrip():
    m = np.random.default_rng(0).standard_normal(12 * 16 * 16)
    np.testing.assert_array_equal(gio.reorder(gio.reorder(m, r2n=True), n2r=True), m)


def test_ud_grade():
    rng = np.random.default_rng(1)
    m = rng.standard_normal(12 * 8 * 8)
    lo = gio.ud_grade(m, 4)
    nest = gio.reorder(m, r2n=True)
    np.testing.assert_allclose(gio.reorder(lo, r2n=True), nest.reshape(-1, 4).mean(axis=1), rtol=1e-14)
    assert lo.mean() == pytest.approx(m.mean(), abs=1e-13)
    up = gio.ud_grade(lo, 8)
    np.testing.assert_array_equal(gio.reorder(up, r2n=True), np.repeat(gio.reorder(lo, r2n=True), 4))
    # UNSEEN children are skipped; pess marks the parent UNSEEN
    nest[:3] = gio.UNSEEN
    m2 = gio.reorder(nest, n2r=True)
    a = gio.reorder(gio.ud_grade(m2, 4), r2n=True)
    b = gio.reorder(gio.ud_grade(m2, 4, pess=True), r2n=True)
    assert a[0] == pytest.approx(nest[3]) and b[0] == gio.UNSEEN
    nest[3] = gio.UNSEEN
    assert gio.reorder(gio.ud_grade(gio.reorder(nest, n2r=True), 4), r2n=True)[0] == gio.UNSEEN
    # a binary mask keeps f_sky on degrading
    th, _ = O.pixel_angles(16)
    mask = (np.abs(np.cos(th)) > 0.2).astype(float)
    assert gio.ud_grade(mask, 4).mean() == pytest.approx(mask.mean(), rel=1e-12)
    np.testing.assert_array_equal(gio.ud_grade(m, 8, order_in="RING", order_out="NESTED"), gio.reorder(m, r2n=True))


@pytest.mark.parametrize("nest", [False, True])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_fits_roundtrip(tmp_path, nest, dtype):
    rng = np.random.default_rng(2)
    maps = rng.standard_normal((3, 12 * 16 * 16)).astype(dtype)
    p = str(tmp_path / "m.fits")
    gio.write_map(p, maps if not nest else gio.reorder(maps, r2n=True), nest=nest, dtype=dtype)
    assert os.path.getsize(p) % 2880 == 0
    got = gio.read_map(p, field=(0, 1, 2))
    np.testing.assert_array_equal(got, maps.astype(np.float64))
    np.testing.assert_array_equal(gio.read_map(p), maps[0].astype(np.float64))
    np.testing.assert_array_equal(gio.read_map(p, 1, nest=True), gio.reorder(maps[1], r2n=True).astype(np.float64))
    _, hdr = gio.read_map(p, h=True)
    hd = dict(hdr)
    assert hd["NSIDE"] == 16 and hd["ORDERING"] == ("NESTED" if nest else "RING") and hd["PIXTYPE"] == "HEALPIX"
    with pytest.raises(OSError):
        gio.write_map(p, maps)


def _hand_fits(path, values_be, tform, extra_cards=()):
    def card(s):
        return s.ljust(80)
    prim = "".join(card(c) for c in ["SIMPLE  =                    T", "BITPIX  =                    8",
                                       "NAXIS   =                    0", "EXTEND  =                    T",
                                       "COMMENT hand-built test file", "END"])
    nrow = 1
    ext = ["XTENSION= 'BINTABLE'", "BITPIX  =                    8", "NAXIS   =                    2",
           "NAXIS1  = %20d" % len(values_be), "NAXIS2  = %20d" % nrow, "PCOUNT  =                    0",
           "GCOUNT  =                    1", "TFIELDS =                    1", "TTYPE1  = 'SIGNAL  '",
           "TFORM1  = '%s'" % tform] + list(extra_cards) + ["PIXTYPE = 'HEALPIX '", "NSIDE   =                    1"]
    if not any(c.startswith("INDXSCHM") for c in extra_cards):
        ext.append("INDXSCHM= 'IMPLICIT'")
    ext.append("END")
    ext = "".join(card(c) for c in ext)
    pad = lambda b: b + b" " * ((-len(b)) % 2880)
    data = values_be + b"\0" * ((-len(values_be)) % 2880)
    with open(path, "wb") as f:
        f.write(pad(prim.encode()) + pad(ext.encode()) + data)


def test_fits_hand_built(tmp_path):
    """a standard-conformant file written byte by byte: big-endian int16
    column with TSCAL/TZERO and TNULL, NESTED ordering, O'Hara-style quoting."""
    vals = np.arange(12, dtype=">i2")
    vals[5] = -32768
    p = str(tmp_path / "h.fits")
    _hand_fits(p, vals.tobytes(), "12I", ["TSCAL1  =                  0.5", "TZERO1  =                  1.0",
                                         "TNULL1  =               -32768", "ORDERING= 'NESTED  '",
                                         "OBJECT  = 'IT''S A MAP'"])
    m, hdr = gio.read_map(p, h=True)
    want = np.arange(12) * 0.5 + 1.0
    want[5] = gio.UNSEEN
    np.testing.assert_array_equal(m, want)          # nside 1: NESTED == RING
    assert dict(hdr)["OBJECT"] == "IT'S A MAP"


def test_fits_errors(tmp_path):
    p = str(tmp_path / "bad.fits")
    _hand_fits(p, np.arange(12, dtype=">f4").tobytes(), "12E", ["INDXSCHM= 'EXPLICIT'"])
    with pytest.raises(NotImplementedError):
        gio.read_map(p)
    _hand_fits(p, np.arange(12, dtype=">f4").tobytes(), "12X")
    with pytest.raises(ValueError):
        gio.read_map(p)


def test_run_record_npz_roundtrip(tmp_path):
    bins = {"EE": np.arange(10), "BB": np.arange(8)}
    blocks = {"EE": np.array([2, 10]), "BB": np.array([2, 5, 6, 7, 8])}
    pv = {"EE": np.ones(7), "BB": np.ones(5) * 2}
    h = {"EE": np.random.default_rng(3).random((4, 9)), "BB": np.random.default_rng(4).random((4, 7))}
    rec = gio.run_record(h, np.ones(3, dtype=int), np.zeros(3), bins, blocks, pv, 1.5, 1.2, pcg_accuracy=1e-5,
                         gibbs_iterations=20, gibbs_cr=True)
    p = str(tmp_path / "run.npz")
    gio.save_npz(p, rec)
    back = gio.load_npz(p)
    assert set(back) == set(rec)
    for k, v in rec.items():
        if isinstance(v, dict):
            for s in v:
                np.testing.assert_array_equal(back[k][s], v[s])
        elif v is None:
            assert back[k] is None
        else:
            np.testing.assert_array_equal(back[k], v)
    ds = gio.dataset_record({"Q": np.ones(12), "U": np.zeros(12)}, np.ones((3, 12)), np.ones((4, 5)), 0.5, 1600.0,
                            0.04, None, 1, 4)
    gio.save_npz(str(tmp_path / "ds.npz"), ds)
    assert gio.load_npz(str(tmp_path / "ds.npz"))["mask_path"] is None
