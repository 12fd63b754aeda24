"""Pin the CPU oracle against golden vectors produced by the reference itself
(tools/gen_golden.py).  Floating point tolerance: 1e-12 relative unless noted."""
import numpy as np
import pytest

from oracle import harmonic as H
from oracle import reference_eb as R
from tests._golden import load, model_from, init_of

RTOL = 1e-12


@pytest.fixture(scope="module")
def g():
    return load(16)


def test_var_expansion_a1(g):
    np.testing.assert_allclose(H.generate_var_cl(g["a1_dl"]), g["a1_var"], rtol=RTOL, atol=0)


def test_layout_a3(g):
    L = int(g["L"])
    c = H.real_to_complex(g["a3_real"], L)
    np.testing.assert_allclose(c.real, g["a3_cplx_re"], rtol=RTOL, atol=1e-15)
    np.testing.assert_allclose(c.imag, g["a3_cplx_im"], rtol=RTOL, atol=1e-15)
    np.testing.assert_allclose(H.complex_to_real(c, L), g["a3_back"], rtol=RTOL, atol=1e-15)


def test_unfold_a5(g):
    np.testing.assert_array_equal(H.unfold_bins(g["a5_binned"], g["bins_BB"]), g["a5_unfold"])


def test_beam_matches_reference(g):
    L = int(g["L"])
    np.testing.assert_allclose(H.gauss_beam(float(g["fwhm_deg"]) * np.pi / 180, L), g["bl_gauss_ref"], rtol=1e-14)


def test_centered_cr_a7(g):
    m = model_from(g)
    np.random.seed(int(g["a7_seed"]))
    s = R.cr_centered(m, np.stack([g["dl_EE"], g["dl_BB"]]))
    np.testing.assert_allclose(s[0], g["a7_E"], rtol=RTOL, atol=1e-13)
    np.testing.assert_allclose(s[1], g["a7_B"], rtol=RTOL, atol=1e-13)


def test_noncentered_cr_a8(g):
    m = model_from(g)
    np.random.seed(int(g["a8_seed"]))
    s = R.cr_noncentered(m, np.stack([g["dl_EE"], g["dl_BB"]]))
    np.testing.assert_allclose(s[0], g["a8_E"], rtol=RTOL, atol=1e-13)
    np.testing.assert_allclose(s[1], g["a8_B"], rtol=RTOL, atol=1e-13)


def test_centered_cls_draw_a13(g):
    m = model_from(g)
    np.random.seed(int(g["a13_seed"]))
    d = R.cls_centered(m, np.stack([g["a7_E"], g["a7_B"]]))
    np.testing.assert_allclose(d["EE"], g["a13_EE"], rtol=1e-10)
    np.testing.assert_allclose(d["BB"], g["a13_BB"], rtol=1e-10)


def test_nc_mh_a15(g):
    m = model_from(g)
    np.random.seed(int(g["a15_seed"]))
    d, acc = R.nc_mh(m, np.stack([g["a8_E"], g["a8_B"]]), init_of(g))
    np.testing.assert_array_equal(acc["EE"], g["a15_acc_EE"])
    np.testing.assert_array_equal(acc["BB"], g["a15_acc_BB"])
    np.testing.assert_allclose(d["EE"], g["a15_EE"], rtol=1e-9)
    np.testing.assert_allclose(d["BB"], g["a15_BB"], rtol=1e-9)


def test_noncentered_driver_a16(g):
    m = model_from(g)
    np.random.seed(int(g["nc_seed"]))
    h, acc, _ = R.run_noncentered(m, init_of(g), int(g["nc_iters"]))
    np.testing.assert_allclose(h["EE"], g["nc_h_EE"], rtol=1e-9)
    np.testing.assert_allclose(h["BB"], g["nc_h_BB"], rtol=1e-9)
    np.testing.assert_array_equal(acc["EE"], g["nc_acc_EE"])


def test_centered_driver_a16(g):
    m = model_from(g)
    np.random.seed(int(g["c_seed"]))
    h, _ = R.run_centered(m, init_of(g), int(g["c_iters"]))
    np.testing.assert_allclose(h["EE"], g["c_h_EE"], rtol=1e-9)
    np.testing.assert_allclose(h["BB"], g["c_h_BB"], rtol=1e-9)


def test_asis_driver_a16(g):
    m = model_from(g)
    np.random.seed(int(g["asis_seed"]))
    h, acc, _ = R.run_asis(m, init_of(g), int(g["asis_iters"]))
    np.testing.assert_allclose(h["EE"], g["asis_h_EE"], rtol=1e-9)
    np.testing.assert_allclose(h["BB"], g["asis_h_BB"], rtol=1e-9)
    np.testing.assert_array_equal(acc["BB"], g["asis_acc_BB"])
