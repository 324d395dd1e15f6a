"""Can two RCCL ranks share the one GPU of a gpurun box?  Two processes, both on cuda:0, one
all_reduce over backend "nccl" (= RCCL).  Prints the result or the error.

    python tools/rccl_two_rank_probe.py
"""
import os
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def worker(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.cuda.set_device(0)
    try:
        dist.init_process_group("nccl", rank=rank, world_size=world)
        x = torch.full((4,), float(rank + 1), device="cuda")
        dist.all_reduce(x)
        torch.cuda.synchronize()
        print(f"rank {rank}: all_reduce -> {x.tolist()}", flush=True)
        dist.destroy_process_group()
    except Exception as e:  # report, do not retry
        print(f"rank {rank}: {type(e).__name__}: {str(e)[:300]}", flush=True)
        sys.exit(3)


if __name__ == "__main__":
    mp.spawn(worker, args=(2, 29631), nprocs=2, join=True)
