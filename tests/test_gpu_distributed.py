"""GPU: the sharded multi-process path end to end through the drop-in surface.
Two ranks (torchrun-style environment, gloo for the host collectives so both
can share the one GPU of the test box) each run NonCenteredGibbs(...,
distributed=True, nchains=2) on the device; run() returns all four global
chains (histories all-gathered) and they equal a single-process 4-chain run:
a chain's trajectory does not depend on the number of ranks."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _sampler(nchains, **kw):
    from gibbssampler_amd import gibbs as G
    from tests._util import make_problem
    m, init = make_problem(40, 16, 2, seed=3)
    smp = G.NonCenteredGibbs({"EE": m.d_alm[0], "BB": m.d_alm[1]}, 40.0 ** 2, 0.2 ** 2, 1.0, 16, 40, 3072,
                             m.proposal_variances, metropolis_blocks=m.blocks, polarization=True, bins=m.bins,
                             n_iter=5, all_sph=True, nchains=nchains, rng="native", seed=31, **kw)
    return smp, init


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK="0")
    smp, init = _sampler(2, distributed=True, dist_backend="gloo")
    h, acc, _, _ = smp.run(init)
    q.put((rank, {s: v for s, v in h.items()}, {s: v for s, v in acc.items()}))
    smp.shard.close()


@pytest.mark.timeout(240)
def test_two_ranks_through_the_surface_equal_one_process():
    import torch.multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=200) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    one, init = _sampler(4)
    h, acc, _, _ = one.run(init)
    for rank, hg, ag in got:
        for s in h:
            assert hg[s].shape == h[s].shape            # [n_iter + 1, 4 global chains, nbins]
            np.testing.assert_array_equal(hg[s], h[s])
            np.testing.assert_array_equal(ag[s], acc[s])
