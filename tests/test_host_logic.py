"""Host-side logic without a GPU: problem / config recipes vs the reference
config, sharding of chains, and the EB golden problem's structure."""
import numpy as np

from gibbssampler_amd import problem
from gibbssampler_amd.distributed import shard_chains


def test_reference_config_recipes_at_512():
    """config.py:45-55: Planck BB bins to 513, 1 EE block, [2, 279] + per-bin BB blocks."""
    bins = problem.default_bins(512, 2)
    assert bins["BB"][-1] == 513 and len(bins["BB"]) == 413
    assert np.array_equal(bins["EE"], np.arange(0, 514))
    blocks = problem.default_blocks(512, bins)
    assert list(blocks["EE"]) == [2, 514]
    assert list(blocks["BB"][:3]) == [2, 279, 280] and blocks["BB"][-1] == 412
    assert len(blocks["BB"]) - 1 == 134


def test_synthetic_problem_shapes():
    P = problem.synthetic_problem(32, 16, 3, seed=0)
    assert P["d_alm"].shape == (3, 33 ** 2)
    assert set(P["bins"]) == {"TT", "EE", "BB", "TE"}
    for s, pv in P["proposal_variances"].items():
        assert len(pv) == len(P["bins"][s]) - 3
        assert np.all(pv > 0)
    assert P["dls_init"]["EE"][0] == 0 and P["dls_init"]["EE"][5] > 0


def test_shard_chains_partition():
    world, k = 8, 32
    owned = [shard_chains(world, r, k) for r in range(world)]
    flat = sorted(c for o in owned for c in o)
    assert flat == list(range(world * k))


def test_unfold_bins_matches_reference_semantics():
    from gibbssampler_amd.utils import unfold_bins
    b = np.array([0, 1, 2, 5, 9])
    np.testing.assert_array_equal(unfold_bins([1.0, 2.0, 3.0, 4.0], b), [1, 2, 3, 3, 3, 4, 4, 4, 4])


def test_graveyard_drains_only_at_explicit_points():
    """entries parked during a capture this package did not open
    (end_capture never runs for it) stay parked through unrelated releases and
    parks -- a graph captured outside the package may still replay kernels that
    use them -- and are freed by the explicit flush()."""
    from gibbssampler_amd import _capi
    freed = []
    _capi._GRAVEYARD.append((freed.append, "handle-a"))       # as if parked inside a foreign capture
    _capi._GRAVEYARD.append((None, object()))
    _capi.release(freed.append, "handle-b")
    assert freed == ["handle-b"] and _capi.graveyard_size() == 2
    assert _capi.park(object()) is False
    assert _capi.graveyard_size() == 2
    _capi.flush()
    assert freed == ["handle-b", "handle-a"] and _capi.graveyard_size() == 0
