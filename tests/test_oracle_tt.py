"""CPU: the temperature-only oracle (oracle/masked.py tt_*) against golden
vectors from the reference's own TT path (tools/gen_golden_tt.py; HEAD's three
missing TT definitions supplied as documented there).  Pins the full-sky
centred / non-centred CRs, the auxiliary-variable CR, the TT C_l draw, the
pixel-likelihood MH sweep (full sky and masked) and the three drivers."""
import os

import numpy as np
import pytest

from oracle import harmonic as H
from oracle import masked as MK
from oracle import reference_eb as RE

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_tt_N8_L16.npz")


@pytest.fixture(scope="module")
def g():
    return dict(np.load(GOLDEN))


def _close(a, b):
    np.testing.assert_allclose(a, b, rtol=1e-10, atol=1e-12 * np.abs(b).max())


def _mm(g, masked=False):
    Npix = int(g["Npix"])
    inv = np.full(Npix, 1.0 / float(g["noise"]))
    if masked:
        inv = inv * g["mask"]
    return MK.tt_model(int(g["L"]), int(g["nside"]), g["bl"], g["T"], inv)


def _model(g):
    L = int(g["L"])
    return H.Model(L, int(g["nside"]), 1, g["bl"], [1.0], {"TT": g["bins"]}, blocks={"TT": g["blocks"]},
                   proposal_variances={"TT": g["pv"]}, d_alm=np.zeros((1, (L + 1) ** 2)))


def _dl(g):
    return g["dl_TT"][None]


def test_fullsky_cr(g):
    mm = _mm(g)
    nr = (int(g["L"]) + 1) ** 2
    for key, nc in (("cr_c", False), ("cr_nc", True)):
        np.random.seed(int(g[key + "_seed"]))
        zs = np.random.normal(size=nr)
        zp = np.random.normal(size=mm.Npix)
        _close(MK.tt_fullsky_cr(mm, _dl(g), zs, zp, noncentered=nc), g[key])


def test_aux(g):
    mm = _mm(g, masked=True)
    assert mm.mu[0] == pytest.approx(float(g["aux_mu"]), rel=1e-15)
    s, acc = MK.aux_variable(mm, _dl(g), g["aux_s_old"][None], 1, MK.ReplayDraws(int(g["aux_seed"])))
    assert acc == int(g["aux_accept"])
    _close(s[0], g["aux_out"])


def test_cls_draw(g):
    np.random.seed(int(g["cls_seed"]))
    out = RE.cls_centered(_model(g), g["cr_c"][None])
    _close(out["TT"], g["cls_out"])


@pytest.mark.parametrize("tag", ["mh", "mhm"])
def test_pixel_mh(g, tag):
    mm = _mm(g, masked=(tag == "mhm"))
    model = _model(g)
    init = {"TT": g["init"].copy()}
    assert MK.nc_loglik_pixel(mm, model.unfold(init), g["mh_snc"][None]) == pytest.approx(float(g[tag + "_lik0"]),
                                                                                          rel=1e-11)
    np.random.seed(int(g[tag + "_seed"]))
    u_prop, u_acc = RE.draw_mh_uniforms(model)
    new, acc = MK.pixel_mh(mm, model, init, g["mh_snc"][None], u_prop=u_prop, u_accept=u_acc)
    _close(new["TT"], g[tag + "_out"])
    assert acc["TT"] == list(g[tag + "_accept"])


@pytest.mark.parametrize("kind,key,gcr", [("centered", "drv_c", False), ("noncentered", "drv_nc", False),
                                          ("asis", "drv_asis", False), ("asis", "drv_asisg", True)])
def test_drivers(g, kind, key, gcr):
    mm = _mm(g)
    np.random.seed(int(g[key + "_seed"]))
    h, acc, _ = MK.tt_chain(kind, mm, mm, _model(g), {"TT": g["init"]}, int(g["drv_iters"]), MK.ReplayDraws(),
                            gibbs_cr=gcr)
    _close(h, g[key + "_h"])
    if kind != "centered":
        np.testing.assert_array_equal(acc, g[key + "_acc"])
