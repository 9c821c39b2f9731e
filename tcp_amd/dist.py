"""One process per GPU: the little distributed plumbing the batch path needs.

Packets are independent, so the data path has no collective:
each rank checksums its own slice in its own HBM.  torch.distributed (RCCL
as "nccl" on the GPU box, gloo in CPU tests) is used only for the
barrier around the timed region and the max-over-ranks time.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import time


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


def launched() -> bool:
    """True when a launcher (torchrun, or spawn_ranks below) set up the ranks."""
    return "WORLD_SIZE" in os.environ


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n: int, argv: list[str], extra_env: dict | None = None, timeout: float | None = None) -> int:
    """Start n rank processes of ``python argv...`` (one per GPU) with the
    torchrun environment (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1,
    MASTER_PORT) and wait for all of them.  Children are started before the
    caller touches any GPU, as separate processes (never exec).  Returns 0 when
    every rank exits 0, else the first nonzero exit status (a rank killed by a
    signal counts as 128 + signal)."""
    port = free_port()
    procs = []
    for r in range(n):
        e = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        e.update(extra_env or {})
        procs.append(subprocess.Popen([sys.executable] + list(argv), env=e))
    # poll every rank (not one after another): a rank that fails while rank 0
    # waits in a barrier must end the others at once, not after a rendezvous
    # time-out
    t0 = time.monotonic()
    rc = 0
    while True:
        codes = [p.poll() for p in procs]
        for code in codes:
            if code:
                code = 128 - code if code < 0 else code
                rc = rc or code
        if rc or all(c is not None for c in codes):
            break
        if timeout is not None and time.monotonic() - t0 > timeout:
            rc = 124
            break
        time.sleep(0.05)
    for q in procs:  # one rank failed or timed out: the others would hang in the next barrier
        if q.poll() is None:
            q.terminate() if rc != 124 else q.kill()
    for q in procs:
        try:
            q.wait(timeout=10)
        except subprocess.TimeoutExpired:
            q.kill()
            q.wait()
    return rc
