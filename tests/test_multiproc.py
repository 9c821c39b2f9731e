"""The N>1 path on CPU with gloo, world_size 2.

Rehearses what bench.py does per rank (its own slice, barrier, max-over-ranks
time) and the byte-balanced strong-scaling split, with the CPU oracle standing
in for the kernel (no GPU here).  Rendezvous on 127.0.0.1.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      LOCAL_RANK=str(rank), WORLD_SIZE=str(world))
    try:
        from oracle import pyoracle
        from tcp_amd import dist as D
        from tcp_amd import workload
        dist = D.init("gloo")
        r, _, w = D.env()
        # weak scaling: every rank its own 1/world of the global index space
        b = workload.make_batch("mixed", rank=r, n=3000)
        host = pyoracle.synth_fill(b.byte_base, b.alloc_bytes, b.seed)
        D.barrier(dist)
        out, flags = pyoracle.batch_ipv4(host, b.descs, nthreads=1)
        t = D.max_over_ranks(dist, 1.0 + r)
        weak = D.gather_objects(dist, (r, b.byte_base, int(out.astype(np.uint64).sum())))
        # strong scaling: one global batch split by bytes
        g = workload.make_batch("mixed", rank=0, n=5000)
        gh = pyoracle.synth_fill(g.byte_base, g.alloc_bytes, g.seed)
        bounds = workload.shard_bounds(g.descs["len"], w)
        part, start, end = workload.rebase(g.descs, int(bounds[r]), int(bounds[r + 1]))
        mine, _ = pyoracle.batch_ipv4(np.ascontiguousarray(gh[start:end + 16]), part, nthreads=1)
        strong = D.gather_objects(dist, (int(bounds[r]), mine.tolist(), int(part["len"].sum())))
        q.put((r, t, weak, strong, None))
        dist.destroy_process_group()
    except Exception as e:  # surfaced in the parent
        q.put((rank, None, None, None, repr(e)))


@pytest.mark.timeout(300)
def test_two_rank_gloo():
    from oracle import pyoracle
    from tcp_amd import workload
    pyoracle.build()
    world, port = 2, free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(60)
    for r, t, weak, strong, err in res:
        assert err is None, err
        assert t == 2.0  # max over ranks
    weak, strong = res[0][2], res[0][3]
    # ranks hold disjoint, consecutive slices of one stream
    assert [w[0] for w in weak] == [0, 1] and weak[1][1] > 0 and weak[1][1] % 16 == 0
    # the strong split covers every packet once, balanced by bytes, and the
    # gathered results equal the single-process batch
    g = workload.make_batch("mixed", rank=0, n=5000)
    gh = pyoracle.synth_fill(g.byte_base, g.alloc_bytes, g.seed)
    full, _ = pyoracle.batch_ipv4(gh, g.descs, nthreads=4)
    joined = np.concatenate([np.array(s[1], np.uint32) for s in sorted(strong)])
    np.testing.assert_array_equal(joined, full)
    b0, b1 = strong[0][2], strong[1][2]
    assert abs(b0 - b1) <= 9000


def test_shard_bounds_balance():
    from tcp_amd import workload
    b = workload.make_batch("mixed", n=100000)
    for world in (1, 2, 3, 4, 8):
        bd = workload.shard_bounds(b.descs["len"], world)
        assert bd[0] == 0 and bd[-1] == b.n and (np.diff(bd) >= 0).all()
        per = [int(b.descs["len"][bd[i]:bd[i + 1]].sum()) for i in range(world)]
        assert max(per) - min(per) <= 2 * 9000
