"""world_size-2 gloo test of the multi-GPU path's host logic on CPU, through the
same functions bench.py and the class surface use (gibbssampler_amd.distributed
.ShardContext): each rank gets its chain offset from the torchrun environment
(and the drop-in NonCenteredGibbs(distributed=True) the same offset), computes
its shard of chains with the (oracle) counter streams, takes the max of its
wall time and all-gathers the traces; the result equals the single-process
computation, i.e. a chain's trajectory does not depend on the GPU count."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _chain_trace(chains, L=12, iters=3):
    from oracle import harmonic as H
    from tests._util import make_problem
    m, init = make_problem(L, 8, 2, seed=3)
    out = np.zeros((iters, len(chains), 2, len(m.bins["EE"]) - 1))
    for j, c in enumerate(chains):
        cur = init
        for it in range(iters):
            un = m.unfold(cur)
            M, Lc = H.noncentered_params(m, un)
            z = np.stack([H.cr_normals(99, c, it, 0, f, L) for f in range(2)])
            s = H.cr_apply_eb_reference(m, M, Lc, m.d_alm, z)
            cur, _ = H.nc_mh(m, cur, H.sweep_stats(m, s, m.d_alm), seed=99, chain=c, iteration=it)
            out[it, j, 0] = cur["EE"]
            out[it, j, 1, :len(cur["BB"])] = cur["BB"]
    return out


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    from gibbssampler_amd.distributed import ShardContext, shard_chains
    from gibbssampler_amd import gibbs as G
    from tests._util import make_problem
    ctx = ShardContext(2, backend="gloo")
    assert (ctx.world, ctx.rank, ctx.chain0, ctx.global_chains) == (world, rank, 2 * rank, 4)
    mine = shard_chains(world, rank, 2)
    assert mine == [ctx.chain0, ctx.chain0 + 1]
    # the drop-in surface takes the same offset from the same context type
    m, init = make_problem(12, 8, 2, seed=3)
    smp = G.NonCenteredGibbs({"EE": m.d_alm[0], "BB": m.d_alm[1]}, 40.0 ** 2, 0.2 ** 2, 1.0, 8, 12, 768,
                             m.proposal_variances, metropolis_blocks=m.blocks, polarization=True, bins=m.bins,
                             n_iter=3, all_sph=True, nchains=2, distributed=True, dist_backend="gloo")
    assert smp.chain0 == ctx.chain0 and smp.shard.global_chains == 4
    t = torch.from_numpy(_chain_trace(mine))
    full = ctx.gather(t)
    slowest = ctx.max(float(rank + 1))
    if rank == 0:
        q.put((full.numpy(), slowest))
    ctx.barrier()
    import torch.distributed as dist
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_rank_gather_equals_single_process():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    full, slowest = q.get(timeout=240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert slowest == 2.0
    ref = _chain_trace(list(range(4)))
    np.testing.assert_array_equal(full, ref)
