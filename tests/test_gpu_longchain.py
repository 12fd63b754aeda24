"""GPU: a long native chain at the headline configuration against the oracle's
same-stream chain (the north_star bar "within 1e-6
relative on sampled C_l means").

BASELINE configs[2] (NonCenteredGibbs TEB all_sph, N_side 512, l_max 1024,
bench.py's synthetic problem, seed 20261015): chains 0-3 of a 4-chain
BatchedRunner run 100 native iterations as ONE captured hipGraph (the bench
path, sky map not stored) and are compared with the oracle's chains 0-3
(oracle/harmonic.py: cr_normals -> cr_apply -> sweep_stats -> nc_mh;
NonCenteredGibbs.py:134-176, 401-445, 546-560), whose trajectory summaries
tools/gen_golden_longchain.py wrote to tests/golden/longchain_nc_teb_L1024_c4.npz
(the oracle takes ~9 minutes for them; the GPU box only compares):
  * the per-bin means of the binned D_l over the 100 iterations: 1e-6 relative
    (every spectrum, every chain -- at the reference's blocking TT / EE / TE are
    single whole-range Metropolis blocks and stay at their start; BB moves:
    ~12.5k accepted blocks per chain);
  * the D_l after iterations 1, 50 and 100: 1e-8 relative;
  * the accept counts per chain and spectrum: exactly.
"""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = os.path.join(ROOT, "tests", "golden", "longchain_nc_teb_L1024_c4.npz")


def test_longchain_means_vs_oracle():
    from gibbssampler_amd.problem import synthetic_problem
    from gibbssampler_amd.samplers import BatchedRunner
    ref = np.load(FIX)
    niter, nch, seed = int(ref["niter"]), int(ref["nchains"]), int(ref["seed"])
    P = synthetic_problem(1024, 512, 3, seed=0)
    r = BatchedRunner(kind="noncentered", lmax=P["lmax"], nside=P["nside"], nfields=3, nchains=nch, bl=P["bl"],
                      noise_var=P["noise_var"], bins=P["bins"], d_alm=P["d_alm"], blocks=P["blocks"],
                      proposal_variances=P["proposal_variances"], rng="native", seed=seed, chain0=0,
                      store_skymap=False)
    r.init(P["dls_init"])
    p = r.plan
    trace = p.zeros(niter, nch, p.nspec, p.maxbins)
    acc = p.zeros(niter, nch, max(p.nacc, 1), dtype=torch.int32)
    r.capture_steps(niter, trace=trace, trace_capacity=niter, accept_trace=acc)
    r.step()
    torch.cuda.synchronize()
    tr = trace.cpu().numpy()
    ac = acc.cpu().numpy()
    snaps = [int(i) for i in ref["snapshot_iterations"]]
    for k, sp in enumerate(p.spectra):
        nb = len(P["bins"][sp]) - 1
        got_mean = tr[:, :, k, :nb].mean(axis=0)
        want = ref[f"mean_{sp}"]
        np.testing.assert_allclose(got_mean, want, rtol=1e-6, atol=1e-300, err_msg=f"mean {sp}")
        for j, it in enumerate(snaps):
            np.testing.assert_allclose(tr[it - 1, :, k, :nb], ref[f"snap_{sp}"][:, j], rtol=1e-8, atol=1e-300,
                                       err_msg=f"{sp} after iteration {it}")
        got_acc = np.array([sum(int(p.split_accept(torch.from_numpy(ac[i]))[sp][c].sum()) for i in range(niter))
                            for c in range(nch)])
        np.testing.assert_array_equal(got_acc, ref[f"accepts_{sp}"], err_msg=f"accepts {sp}")
    assert int(ref["accepts_BB"].min()) > 1000
