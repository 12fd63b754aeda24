"""Chain sharding across GPUs (one process per GPU, torch.distributed / RCCL).

The reference scales only as independent SLURM array tasks (job-script.sh:6-8);
here a node's GPUs each run a contiguous block of chains of one global run:
rank r owns global chains [r*K, (r+1)*K).  RNG streams are keyed by the
global chain id, so a chain's trajectory does not depend on the GPU count.
No collective runs inside an iteration; the D_l traces are gathered once
(one all_gather over RCCL/xGMI, or gloo on CPU).

One code path for every caller: ``bench.py`` and the ``gibbs.py`` class
surface (``distributed=True``) both use ``ShardContext``.
"""
import os


def dist_env():
    """(world_size, rank, local_rank) from the torchrun environment."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(nproc, script, args, env=None, timeout=None, cwd=None):
    """Run ``script args`` as ``nproc`` ranks of one node under
    ``python -m torch.distributed.run`` (rendezvous on 127.0.0.1), as a child
    process, and return (rank 0's last JSON line as a dict, the child's stdout).
    The caller must not have initialised the GPU (the ranks own it); this
    process only waits.  Raises RuntimeError when the ranks fail or rank 0
    prints no JSON line."""
    import json
    import subprocess
    import sys
    e = dict(os.environ if env is None else env)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
              "GROUP_RANK", "ROLE_RANK", "TORCHELASTIC_RUN_ID"):
        e.pop(k, None)
    e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={int(nproc)}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", script] + [str(a) for a in args]
    out = subprocess.run(cmd, env=e, cwd=cwd, stdout=subprocess.PIPE, text=True, timeout=timeout)
    if out.returncode != 0:
        raise RuntimeError(f"launch_ranks: {nproc} ranks of {script} exited with {out.returncode}")
    line = None
    for ln in out.stdout.splitlines():
        ln = ln.strip()
        if ln.startswith("{"):
            try:
                line = json.loads(ln)
            except ValueError:
                pass
    if line is None:
        raise RuntimeError(f"launch_ranks: rank 0 of {script} printed no JSON line")
    return line, out.stdout


def shard_chains(world_size, rank, chains_per_rank):
    """Global chain ids owned by ``rank``."""
    if not (0 <= rank < world_size):
        raise ValueError("rank out of range")
    c0 = rank * chains_per_rank
    return list(range(c0, c0 + chains_per_rank))


class ShardContext:
    """The run's place in a torchrun job: world size, rank, local GPU, the
    first global chain of this rank, and the three host-side collectives the
    run needs (barrier, max of a scalar, trace gather).  world_size 1 without
    torch.distributed is the single-process case (every call is local).

    backend: "nccl" (RCCL, one GPU per rank) or "gloo" (CPU; tests)."""

    def __init__(self, chains_per_rank, backend="nccl", init=True):
        import torch
        import torch.distributed as dist
        self.world, self.rank, self.local = dist_env()
        self.chains_per_rank = int(chains_per_rank)
        self.chain0 = self.rank * self.chains_per_rank
        self.backend = backend
        self.device = torch.device("cuda", self.local) if backend == "nccl" else torch.device("cpu")
        self._owns_group = False
        if self.world > 1:
            if not dist.is_initialized():
                if not init:
                    raise RuntimeError("WORLD_SIZE > 1 but torch.distributed is not initialised")
                kw = {"device_id": self.device} if backend == "nccl" else {}
                dist.init_process_group(backend, **kw)
                self._owns_group = True
            if dist.get_world_size() != self.world:
                raise RuntimeError("WORLD_SIZE does not match the process group")
        elif dist.is_available() and dist.is_initialized():
            # a group the caller initialised (any size, e.g. one RCCL rank on a
            # one-GPU box): its collectives are used as for world > 1
            if dist.get_world_size() != self.world:
                raise RuntimeError("WORLD_SIZE does not match the process group")
        grouped = self.world > 1 or (dist.is_available() and dist.is_initialized())
        self.dist = dist if grouped else None

    @property
    def global_chains(self):
        return self.world * self.chains_per_rank

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def max(self, value):
        """max over ranks of a host float (the timed region's wall time)."""
        if self.dist is None:
            return float(value)
        import torch
        t = torch.tensor([float(value)], dtype=torch.float64, device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def gather(self, trace, dim=1):
        """all_gather a per-rank tensor and concatenate along ``dim`` (the chain
        axis) in rank order = global chain order."""
        if self.dist is None:
            return trace
        import torch
        dev = trace.device
        t = trace.contiguous()
        if self.backend == "gloo" and t.is_cuda:
            t = t.cpu()                      # gloo gathers host tensors
        parts = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(parts, t)
        return torch.cat(parts, dim=dim).to(dev)

    def close(self):
        if self.dist is not None and self._owns_group:
            self.dist.barrier()
            self.dist.destroy_process_group()
            self._owns_group = False

