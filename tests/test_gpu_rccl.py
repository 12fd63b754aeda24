"""GPU: the sharded path over RCCL itself.  The test box has one GPU, so the
process group is one rank with the "nccl" backend (RCCL) bound to cuda:0:
ShardContext's barrier, max and trace all_gather then run as RCCL
collectives on device tensors, and a run through the drop-in surface with
distributed=True, dist_backend="nccl" equals the same run without the group.
(Multi-rank RCCL needs one GPU per rank: the driver's 8-GPU scaling bench.)"""
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


def _sampler(**kw):
    from gibbssampler_amd import gibbs as G
    from tests._util import make_problem
    m, init = make_problem(40, 16, 2, seed=3)
    smp = G.NonCenteredGibbs({"EE": m.d_alm[0], "BB": m.d_alm[1]}, 40.0 ** 2, 0.2 ** 2, 1.0, 16, 40, 3072,
                             m.proposal_variances, metropolis_blocks=m.blocks, polarization=True, bins=m.bins,
                             n_iter=5, all_sph=True, nchains=3, rng="native", seed=31, **kw)
    return smp, init


def _worker(port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    from gibbssampler_amd.distributed import ShardContext
    sc = ShardContext(3, backend="nccl")
    assert sc.dist is not None                     # the RCCL group is used
    sc.barrier()
    mx = sc.max(2.5)
    g = sc.gather(torch.arange(6, dtype=torch.float64, device="cuda").reshape(2, 3), dim=1)
    smp, init = _sampler(distributed=True, dist_backend="nccl")
    h, acc, _, _ = smp.run(init)
    q.put((dist.get_backend(), mx, g.cpu().numpy(), {s: v for s, v in h.items()}, {s: v for s, v in acc.items()}))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(240)
def test_rccl_group_collectives_and_surface_run():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    backend, mx, g, hg, ag = q.get(timeout=200)
    p.join(60)
    assert p.exitcode == 0
    assert backend == "nccl"
    assert mx == 2.5
    np.testing.assert_array_equal(g, np.arange(6, dtype=np.float64).reshape(2, 3))
    one, init = _sampler()
    h, acc, _, _ = one.run(init)
    for s in h:
        np.testing.assert_array_equal(hg[s], h[s])
        np.testing.assert_array_equal(ag[s], acc[s])
