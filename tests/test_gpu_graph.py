"""GPU: hipGraph-captured steps (samplers.BatchedRunner.capture_graph) give
bit-identical chains to eager steps -- the NC graph fuses the trace record
and the counter advance into the MH decision launch, the centered graph into
the C_l-draw launch (gs_step_centered_fused), the ASIS graph into its MH
launch (gs_step_asis_fused)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _runner(kind, F, nchains=4):
    from gibbssampler_amd.problem import synthetic_problem
    from gibbssampler_amd.samplers import BatchedRunner
    P = synthetic_problem(64, 32, F, seed=3)
    r = BatchedRunner(kind, P["lmax"], P["nside"], P["nfields"], nchains, P["bl"], P["noise_var"], P["bins"],
                      P["d_alm"], blocks=P["blocks"], proposal_variances=P["proposal_variances"], rng="native",
                      seed=91, chain0=2)
    r.init(P["dls_init"])
    return r


@pytest.mark.parametrize("kind,F", [("noncentered", 3), ("noncentered", 2), ("noncentered", 1),
                                    ("centered", 3), ("centered", 2), ("centered", 1), ("asis", 2), ("asis", 3)])
def test_graph_equals_eager(kind, F):
    import torch
    n, w = 6, 2
    eager = _runner(kind, F)
    want, wacc = [], []
    for _ in range(w + n):
        eager.step()
        want.append(eager.dl.cpu().numpy().copy())
        wacc.append(eager.accept.cpu().numpy().copy())
    g = _runner(kind, F)
    for _ in range(w):
        g.step()
    p = g.plan
    trace = p.zeros(n, p.nchains, p.nspec, p.maxbins)
    g.capture_graph(trace=trace, trace_capacity=n)
    got_acc = []
    for _ in range(n):
        g.step()
        got_acc.append(g.accept.cpu().numpy().copy())
    torch.cuda.synchronize()
    tr = trace.cpu().numpy()
    # the trace slot of iteration it is (it - 1) % n; iterations w+1 .. w+n
    for k in range(n):
        it = w + 1 + k
        np.testing.assert_array_equal(tr[(it - 1) % n], want[w + k])
    np.testing.assert_array_equal(g.dl.cpu().numpy(), want[-1])
    if kind != "centered":
        np.testing.assert_array_equal(np.array(got_acc), np.array(wacc[w:]))
    # after the graph, eager steps continue the same chains
    g.graph = None
    p.iteration_counter(False)
    g.step()
    eager.step()
    np.testing.assert_array_equal(g.dl.cpu().numpy(), eager.dl.cpu().numpy())


@pytest.mark.parametrize("kind,F", [("noncentered", 3), ("noncentered", 2), ("centered", 3), ("asis", 3)])
def test_multistep_graph_with_sweep_timing(kind, F):
    """bench.py's timed region: K iterations in ONE graph with the sweeps
    bracketed by captured event nodes -- same chains as eager, K timings."""
    import torch
    n, w = 5, 2
    eager = _runner(kind, F)
    want = []
    for _ in range(w + n):
        eager.step()
        want.append(eager.dl.cpu().numpy().copy())
    g = _runner(kind, F)
    for _ in range(w):
        g.step()
    p = g.plan
    trace = p.zeros(n, p.nchains, p.nspec, p.maxbins)
    g.capture_steps(n, trace=trace, trace_capacity=n, time_sweeps=True, time_every=2)
    g.step()
    torch.cuda.synchronize()
    ms, cnt = p.sweep_timing(False)
    assert cnt == (n + 1) // 2 and ms > 0
    tr = trace.cpu().numpy()
    for k in range(n):
        it = w + 1 + k
        np.testing.assert_array_equal(tr[(it - 1) % n], want[w + k])
    np.testing.assert_array_equal(g.dl.cpu().numpy(), want[-1])
    assert g.iteration == w + n
