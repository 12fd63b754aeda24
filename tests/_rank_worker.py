"""Stand-in rank program for tests/test_launch_cpu.py: what bench.py's ranks do
around their timed region (gloo process group from the torchrun environment,
a max over ranks, rank 0 prints one JSON line), without a GPU."""
import json
import os
import sys

import torch
import torch.distributed as dist


def main():
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    dist.init_process_group("gloo")
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ranks = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(ranks, torch.tensor([rank], dtype=torch.int64))
    gpus = int(sys.argv[sys.argv.index("--gpus") + 1]) if "--gpus" in sys.argv else 1
    if rank == 0:
        print(json.dumps({"metric": "stand-in", "value": float(t.item()), "n_gpus": world, "gpus_arg": gpus,
                          "ranks_seen": [int(r.item()) for r in ranks], "cpu_baseline": None,
                          "argv": sys.argv[1:]}))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
