"""Chain sharding across GPUs (one process per GPU, torch.distributed / RCCL).

The reference scales only as independent SLURM array tasks (job-script.sh:6-8);
here a node's GPUs each run a contiguous block of chains of one global run:
rank r owns global chains [r*K, (r+1)*K).  RNG streams are keyed by the
global chain id, so a chain's trajectory does not depend on the GPU count.
No collective runs inside an iteration; the D_l traces are gathered once
(``gather_traces``: one all_gather over RCCL/xGMI, or gloo on CPU).
"""
import os


def dist_env():
    """(world_size, rank, local_rank) from the torchrun environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard_chains(world_size, rank, chains_per_rank):
    """Global chain ids owned by ``rank``."""
    if not (0 <= rank < world_size):
        raise ValueError("rank out of range")
    c0 = rank * chains_per_rank
    return list(range(c0, c0 + chains_per_rank))


def gather_traces(trace, group=None):
    """All-gather a per-rank trace tensor [n_iter, chains_per_rank, ...] into
    [n_iter, world * chains_per_rank, ...] ordered by global chain id."""
    import torch
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        return trace
    world = dist.get_world_size(group)
    parts = [torch.empty_like(trace) for _ in range(world)]
    dist.all_gather(parts, trace.contiguous(), group=group)
    return torch.cat(parts, dim=1)
