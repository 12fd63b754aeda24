"""The reference class surface (gibbssampler_amd.gibbs) and utils on the GPU,
checked against the reference goldens (replay mode)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from tests._golden import load, init_of  # noqa: E402


@pytest.fixture(scope="module")
def g():
    return load(16)


def _args(g):
    Npix = int(g["Npix"])
    pix_map = {"EE": g["d_E"], "BB": g["d_B"], "Q": np.zeros(Npix), "U": np.zeros(Npix)}
    return pix_map, np.ones(Npix) * float(g["noise_temp"]), np.ones(Npix) * float(g["noise_pol"]), Npix


def test_noncentered_gibbs_surface(g):
    from gibbssampler_amd.gibbs import NonCenteredGibbs
    pix_map, nt, npol, Npix = _args(g)
    bins = {"EE": g["bins_EE"], "BB": g["bins_BB"]}
    ncg = NonCenteredGibbs(pix_map, nt, npol, float(g["fwhm_deg"]), int(g["nside"]), int(g["L"]), Npix,
                           proposal_variances={"EE": g["pv_EE"], "BB": g["pv_BB"]},
                           metropolis_blocks={"EE": g["blocks_EE"], "BB": g["blocks_BB"]}, polarization=True,
                           bins=bins, n_iter=int(g["nc_iters"]), all_sph=True, rng="replay")
    np.random.seed(int(g["nc_seed"]))
    h, acc, _, _ = ncg.run(init_of(g))
    np.testing.assert_allclose(h["EE"], g["nc_h_EE"], rtol=1e-9)
    np.testing.assert_allclose(h["BB"], g["nc_h_BB"], rtol=1e-9)
    np.testing.assert_array_equal(acc["BB"], g["nc_acc_BB"])


def test_centered_and_asis_surface(g):
    from gibbssampler_amd.gibbs import CenteredGibbs, ASIS
    pix_map, nt, npol, Npix = _args(g)
    bins = {"EE": g["bins_EE"], "BB": g["bins_BB"]}
    cg = CenteredGibbs(pix_map, nt, npol, float(g["fwhm_deg"]), int(g["nside"]), int(g["L"]), Npix,
                       polarization=True, bins=bins, n_iter=int(g["c_iters"]), rng="replay")
    np.random.seed(int(g["c_seed"]))
    h, acc_cr, _, _ = cg.run(init_of(g))
    np.testing.assert_allclose(h["EE"], g["c_h_EE"], rtol=1e-9)
    np.testing.assert_allclose(h["BB"], g["c_h_BB"], rtol=1e-9)
    asis = ASIS(pix_map, nt, npol, float(g["fwhm_deg"]), int(g["nside"]), int(g["L"]), Npix,
                {"EE": g["pv_EE"], "BB": g["pv_BB"]}, metropolis_blocks={"EE": g["blocks_EE"], "BB": g["blocks_BB"]},
                polarization=True, bins=bins, n_iter=int(g["asis_iters"]), all_sph=True, rng="replay")
    np.random.seed(int(g["asis_seed"]))
    res = asis.run(init_of(g))
    assert len(res) == 7
    np.testing.assert_allclose(res[0]["EE"], g["asis_h_EE"], rtol=1e-9)
    np.testing.assert_allclose(res[0]["BB"], g["asis_h_BB"], rtol=1e-9)


def test_step_samplers_surface(g):
    """constrained_sampler.sample / cls_sampler.sample as the reference drivers call them."""
    from gibbssampler_amd.gibbs import CenteredGibbs, NonCenteredGibbs
    pix_map, nt, npol, Npix = _args(g)
    L = int(g["L"])
    unb = {"EE": np.arange(L + 2), "BB": np.arange(L + 2)}
    cg = CenteredGibbs(pix_map, nt, npol, float(g["fwhm_deg"]), int(g["nside"]), L, Npix, polarization=True,
                       bins={"EE": g["bins_EE"], "BB": g["bins_BB"]}, rng="replay")
    np.random.seed(int(g["a7_seed"]))
    s, acc = cg.constrained_sampler.sample({"EE": g["dl_EE"], "BB": g["dl_BB"]})
    assert acc == 1
    np.testing.assert_allclose(s["EE"], g["a7_E"], rtol=1e-12, atol=1e-13)
    np.random.seed(int(g["a13_seed"]))
    d = cg.cls_sampler.sample({"EE": g["a7_E"], "BB": g["a7_B"]})
    np.testing.assert_allclose(d["BB"], g["a13_BB"], rtol=1e-10)
    ncg = NonCenteredGibbs(pix_map, nt, npol, float(g["fwhm_deg"]), int(g["nside"]), L, Npix,
                           {"EE": g["pv_EE"], "BB": g["pv_BB"]},
                           metropolis_blocks={"EE": g["blocks_EE"], "BB": g["blocks_BB"]}, polarization=True,
                           bins={"EE": g["bins_EE"], "BB": g["bins_BB"]}, all_sph=True, rng="replay")
    np.random.seed(int(g["a8_seed"]))
    s8, a8 = ncg.constrained_sampler.sample({"EE": g["dl_EE"], "BB": g["dl_BB"]})
    assert a8 == 0
    np.testing.assert_allclose(s8["BB"], g["a8_B"], rtol=1e-12, atol=1e-13)
    np.random.seed(int(g["a15_seed"]))
    d15, a15 = ncg.cls_sampler.sample({"EE": g["a8_E"], "BB": g["a8_B"]}, init_of(g))
    np.testing.assert_allclose(d15["BB"], g["a15_BB"], rtol=1e-9)
    assert a15["BB"] == list(g["a15_acc_BB"])
    del unb


def test_utils_surface(g):
    from gibbssampler_amd import utils
    np.testing.assert_allclose(utils.generate_var_cl(g["a1_dl"]), g["a1_var"], rtol=1e-15)
    c = utils.real_to_complex(g["a3_real"])
    np.testing.assert_allclose(c.real, g["a3_cplx_re"], rtol=1e-15, atol=1e-300)
    np.testing.assert_allclose(utils.complex_to_real(c), g["a3_back"], rtol=1e-15)
    np.testing.assert_array_equal(utils.unfold_bins(g["a5_binned"], g["bins_BB"]), g["a5_unfold"])
