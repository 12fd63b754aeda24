"""Oracle vs the reference at the reference's OWN default configuration (CPU).

tests/golden/reference_eb_scale_L512.npz was produced by tools/gen_golden_scale.py
running the reference's Python at N_side 256 / L 512 with config.py's Planck BB
bins, its 1 EE + 134 BB Metropolis blocks and its proposal variances
(config.py:19-21,45-55,119-132,192-197).  The data d is regenerated here from
the fixture's seed (tests/_golden.scale_data).  Tolerance: 1e-9 relative on the
D_l histories (north_star bar: 1e-6 on sampled C_l), accept flags exact.
"""
import numpy as np
import pytest

from oracle import harmonic as H
from oracle import reference_eb as R
from tests._golden import GOLDEN, scale_model


@pytest.fixture(scope="module")
def gs():
    import os
    return dict(np.load(os.path.join(GOLDEN, "reference_eb_scale_L512.npz")))


def test_scale_fixture_is_the_reference_config(gs):
    L = int(gs["L"])
    assert L == 512 and int(gs["nside"]) == 256
    assert len(gs["bins_BB"]) - 1 == 412 and gs["bins_BB"][-1] == 513
    assert len(gs["blocks_EE"]) - 1 == 1 and len(gs["blocks_BB"]) - 1 == 134
    assert len(gs["pv_EE"]) == len(gs["bins_EE"]) - 3 and len(gs["pv_BB"]) == len(gs["bins_BB"]) - 3
    m, D = scale_model(gs)
    np.testing.assert_allclose([D["d_E"].sum(), D["d_B"].sum(), (D["d_E"] ** 2).sum()], gs["d_checksum"],
                               rtol=1e-13)


def test_scale_single_crs(gs):
    m, D = scale_model(gs)
    un = np.stack([D["dl_EE"], D["dl_BB"]])
    for key, params in (("a7", H.centered_params), ("a8", H.noncentered_params)):
        np.random.seed(int(gs[key + "_seed"]))
        M, Lc = params(m, un)
        s = H.cr_apply_eb_reference(m, M, Lc, m.d_alm, R.draw_cr_normals(m))
        np.testing.assert_allclose(s[0, :2048], gs[key + "_head_E"], rtol=1e-12, atol=1e-15)
        np.testing.assert_allclose(s[1, :2048], gs[key + "_head_B"], rtol=1e-12, atol=1e-15)
        np.testing.assert_allclose(H.alm2cl_real(s[0]), gs[key + "_cl_E"], rtol=1e-11)
        np.testing.assert_allclose(H.alm2cl_real(s[1]), gs[key + "_cl_B"], rtol=1e-11)


def _init(gs):
    return {"EE": gs["init_EE"].copy(), "BB": gs["init_BB"].copy()}


def test_scale_noncentered_run(gs):
    m, _ = scale_model(gs)
    np.random.seed(int(gs["nc_seed"]))
    h, acc, _ = R.run_noncentered(m, _init(gs), int(gs["nc_iters"]))
    for s in ("EE", "BB"):
        np.testing.assert_allclose(h[s], gs["nc_h_" + s], rtol=1e-9)
        np.testing.assert_array_equal(acc[s], gs["nc_acc_" + s])


def test_scale_centered_run(gs):
    m, _ = scale_model(gs)
    np.random.seed(int(gs["c_seed"]))
    h, _ = R.run_centered(m, _init(gs), int(gs["c_iters"]))
    for s in ("EE", "BB"):
        np.testing.assert_allclose(h[s], gs["c_h_" + s], rtol=1e-9)


def test_scale_asis_run(gs):
    m, _ = scale_model(gs)
    np.random.seed(int(gs["asis_seed"]))
    out = R.run_asis(m, _init(gs), int(gs["asis_iters"]))
    h, acc = out[0], out[1]
    for s in ("EE", "BB"):
        np.testing.assert_allclose(h[s], gs["asis_h_" + s], rtol=1e-9)
        np.testing.assert_array_equal(acc[s], gs["asis_acc_" + s])
