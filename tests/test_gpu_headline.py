"""The bench line's exact kernel configuration, pinned.

bench.py's default line runs BASELINE configs[2] (NonCenteredGibbs TEB all_sph,
N_side 512, L 1024, 32 chains) through BatchedRunner.capture_steps with the sky
map NOT stored (``k_cr_sweep<3,0,false,0>``).  This test runs that exact path
for 3 iterations and checks:
  * the D_l trace and every accept flag are bit-identical to the same runner
    with the map stored (``store_skymap=True``: the variant every other test
    exercises), and the stored runner's last map reproduces the statistics;
  * chains 0 and 31 of iteration 1 equal the oracle (oracle/harmonic.py:
    cr_apply -> sweep_stats -> nc_mh; NonCenteredGibbs.py:134-176, 401-445):
    D_l at 1e-10 relative, accept flags exactly.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import harmonic as H  # noqa: E402

pytestmark = pytest.mark.gpu

SEED = 20261015
NSTEPS = 3


def _runner(P, store):
    from gibbssampler_amd.samplers import BatchedRunner
    return BatchedRunner(kind="noncentered", lmax=P["lmax"], nside=P["nside"], nfields=3, nchains=32, bl=P["bl"],
                         noise_var=P["noise_var"], bins=P["bins"], d_alm=P["d_alm"], blocks=P["blocks"],
                         proposal_variances=P["proposal_variances"], rng="native", seed=SEED, chain0=0,
                         store_skymap=store)


def _bench_path(runner, P):
    """bench.run_harmonic's graph path: init, the timed steps as ONE captured
    graph with the device D_l trace and a per-step accept trace, one replay."""
    p = runner.plan
    runner.init(P["dls_init"])
    trace = p.zeros(NSTEPS, p.nchains, p.nspec, p.maxbins)
    acc = p.zeros(NSTEPS, p.nchains, max(p.nacc, 1), dtype=torch.int32)
    runner.capture_steps(NSTEPS, trace=trace, trace_capacity=NSTEPS, accept_trace=acc)
    runner.step()
    torch.cuda.synchronize()
    return trace.cpu().numpy(), acc.cpu().numpy()


@pytest.fixture(scope="module")
def problem():
    from gibbssampler_amd.problem import synthetic_problem
    return synthetic_problem(1024, 512, 3, seed=0)


def test_headline_nostore_equals_store_and_oracle(problem):
    P = problem
    r0 = _runner(P, store=False)
    assert r0.s is None
    tr0, ac0 = _bench_path(r0, P)
    nacc = r0.plan.nacc
    del r0
    r1 = _runner(P, store=True)
    tr1, ac1 = _bench_path(r1, P)
    # bit-identical trajectories: the store is the only difference in the kernel
    np.testing.assert_array_equal(tr0, tr1)
    np.testing.assert_array_equal(ac0, ac1)
    assert nacc > 400
    # the oracle at iteration 1 for chains 0 and 31 (the trace rows are the D_l
    # after each iteration's MH; row 0 = iteration 1 from the start D_l)
    m = H.Model(P["lmax"], P["nside"], 3, P["bl"], P["noise_var"], P["bins"], P["blocks"],
                P["proposal_variances"], P["d_alm"])
    un = m.unfold(P["dls_init"])
    M, Lc = H.noncentered_params(m, un)
    p = r1.plan
    spectra = p.spectra
    for c in (0, 31):
        z = np.stack([H.cr_normals(SEED, c, 1, 0, f, m.L) for f in range(3)])
        ref_s = H.cr_apply(m, M, Lc, m.d_alm, z)
        stats = H.sweep_stats(m, ref_s, m.d_alm)
        del ref_s, z
        ref, racc = H.nc_mh(m, P["dls_init"], stats, seed=SEED, chain=c, iteration=1)
        for k, sp in enumerate(spectra):
            nb = len(P["bins"][sp]) - 1
            np.testing.assert_allclose(tr0[0, c, k, :nb], ref[sp], rtol=1e-10, err_msg=f"chain {c} {sp}")
        got = p.split_accept(torch.from_numpy(ac0[0]))
        for sp in spectra:
            np.testing.assert_array_equal(got[sp][c], racc[sp], err_msg=f"chain {c} {sp}")
