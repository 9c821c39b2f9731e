"""One process per GPU: the little distributed plumbing the batch path needs.

Packets are independent, so the data path has no collective:
each rank checksums its own slice in its own HBM.  torch.distributed (RCCL
as "nccl" on the GPU box, gloo in CPU tests) is used only for the
barrier around the timed region and the max-over-ranks time.
"""
from __future__ import annotations

import os


def env():
    """(rank, local_rank, world) from the torchrun environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0")),
            int(os.environ.get("WORLD_SIZE", "1")))


def init(backend: str, local_rank: int | None = None):
    """Initialise the process group when WORLD_SIZE > 1; returns the module or None."""
    rank, local, world = env()
    if world <= 1:
        return None
    import torch
    import torch.distributed as dist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend == "nccl":
        dev = torch.device("cuda", local if local_rank is None else local_rank)
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group(backend)
    return dist


def barrier(dist) -> None:
    if dist is not None:
        dist.barrier()


def max_over_ranks(dist, value: float, device="cpu") -> float:
    if dist is None:
        return value
    import torch
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_objects(dist, obj):
    if dist is None:
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out
