"""tcsum_host_batch_peso's copy / launch plan, checked without a device
(replay the failing fuzz seed's descriptor set through the
host-side planner).  tcsum_debug_plan_host_peso returns the copies and kernels
the call would queue; for every batch of the GPU fuzz test's 32 seeds
(tests/test_gpu_hostq.py::test_host_paths_fuzz) and for extra shapes --
shuffled, sparse, a lead followed by a far-away rest, tiny and empty
segments, every chunk size knob -- the plan must keep each copy inside the
caller's arena and its device buffer, have every byte a kernel reads (its
16-byte chunks) inside the buffer and every byte it sums copied before it,
and launch on every segment exactly once."""
import ctypes

import numpy as np
import pytest

from tcp_amd import _lib
from tcp_amd.csum import PESO_DTYPE


def plan(segs: np.ndarray, arena_bytes: int):
    L = _lib.lib()
    segs = np.ascontiguousarray(segs)
    bufs = np.zeros(2, np.uint64)
    k = L.tcsum_debug_plan_host_peso(segs.ctypes.data, segs.size, arena_bytes, None, 0, bufs.ctypes.data)
    assert k > 0, k
    rows = np.zeros((k, 5), np.uint64)
    k2 = L.tcsum_debug_plan_host_peso(segs.ctypes.data, segs.size, arena_bytes, rows.ctypes.data, k,
                                      bufs.ctypes.data)
    assert k2 == k
    return rows.astype(np.int64), bufs.astype(np.int64)


def check_plan(segs: np.ndarray, arena_bytes: int):
    rows, bufs = plan(segs, arena_bytes)
    off = segs["offset"].astype(np.int64)
    ln = segs["len"].astype(np.int64)
    copied = {0: [], 1: []}  # per buffer: host ranges queued so far
    covered = np.zeros(segs.size, np.int64)
    next_i = 0
    for kind, buf, a, b, c in rows.tolist():
        if kind == 0:  # copy host [a, b) to buffer offset c
            assert 0 <= a < b <= arena_bytes, (a, b, arena_bytes)
            assert 0 <= c and c + (b - a) <= bufs[buf], (c, b - a, bufs[buf])
            copied[buf].append((a, b, c))
            continue
        # kernel on segments [a, b) of buffer `buf` whose byte 0 is arena offset c
        # (kind 2: out of offset order, so the per-range kernel, not the packed stream)
        o_all = off[a:b][ln[a:b] > 0]
        assert (kind == 1) == bool((np.diff(o_all) >= 0).all()), (kind, a, b)
        assert a == next_i and b > a, (a, b, next_i)
        next_i = b
        covered[a:b] += 1
        o, n_ = off[a:b], ln[a:b]
        live = n_ > 0
        lo = (o[live] & ~15) - c
        hi = ((o[live] + n_[live] + 15) & ~15) - c
        assert (lo >= 0).all() and (hi <= bufs[buf]).all(), (lo.min(), hi.max(), bufs[buf])
        # every summed byte copied into this buffer, at the offset the kernel reads it from
        rng = sorted((x, y) for x, y, z in copied[buf] if z == x - c)
        assert len(rng) == len(copied[buf]), "a copy lands at another offset than the kernel reads"
        starts = np.array([x for x, _ in rng])
        ends = np.array([y for _, y in rng])
        j = np.searchsorted(starts, o[live], side="right") - 1
        assert (j >= 0).all()
        assert (ends[j] >= o[live] + n_[live]).all(), "a segment's bytes were not copied before its kernel"
    assert next_i == segs.size and (covered == 1).all()
    return rows, bufs


def fuzz_case(seed: int):
    """The peso batch of test_host_paths_fuzz[seed] (same RNG calls)."""
    rng = np.random.default_rng(1000 + seed)
    n = int(rng.choice([1, 7, 50, 1000, 20000, 60000]))
    layout = rng.choice(["packed", "gaps", "shuffled", "sparse"])
    rng.choice(["pinned", "registered", "pageable"])
    rng.choice(["0", "1", "262144"])
    chunk_mb = int(rng.choice(["1", "8", "64"]))
    lens = rng.integers(0, 3000, n) if rng.random() < 0.5 else rng.integers(20, 9001, n)
    gap = {"gaps": rng.integers(0, 64, n),
           "sparse": rng.integers(0, (1 << 16) if n <= 1000 else 4096, n)}.get(layout, np.zeros(n, np.int64))
    offs = 5 + np.concatenate([[0], np.cumsum(lens + gap)[:-1]]).astype(np.int64)
    arena_bytes = int(offs[-1] + lens[-1] + 32)
    perm = rng.permutation(n) if layout == "shuffled" else np.arange(n)
    segs = np.zeros(n, PESO_DTYPE)
    segs["offset"], segs["len"] = offs[perm], lens[perm]
    return segs, arena_bytes, chunk_mb


@pytest.fixture
def chunk_knob():
    L = _lib.lib()
    yield lambda mb: L.tcsum_debug_set(b"e2e_chunk_mb", int(mb))
    L.tcsum_debug_set(b"e2e_chunk_mb", -1)


@pytest.mark.parametrize("seed", range(32))
def test_fuzz_seed_plans_stay_in_bounds(seed, chunk_knob):
    segs, arena_bytes, chunk_mb = fuzz_case(seed)
    chunk_knob(chunk_mb)
    check_plan(segs, arena_bytes)
    chunk_knob(-1)
    check_plan(segs, arena_bytes)


def test_seed26_plan(chunk_knob):
    """The batch round 4's suite stopped on: 1,000 packed segments of 0..2,999
    bytes from offset 5 (a 1.5-MB pageable arena), 8-MiB chunks -- one copy
    of the span into the arena buffer, one kernel."""
    segs, arena_bytes, chunk_mb = fuzz_case(26)
    assert segs.size == 1000 and chunk_mb == 8
    chunk_knob(chunk_mb)
    rows, bufs = check_plan(segs, arena_bytes)
    assert rows[:, 0].tolist() == [0, 1] and bufs[0] == 0  # in order: the packed stream


@pytest.mark.parametrize("shape", ["lead_then_far", "shuffled_big", "sparse_tail", "zeros", "one_byte_end",
                                   "dense_many_chunks"])
@pytest.mark.parametrize("chunk_mb", [-1, 1, 64])
def test_shapes_plans_stay_in_bounds(shape, chunk_mb, chunk_knob):
    rng = np.random.default_rng(hash(shape) & 0xFFFF)
    if shape == "lead_then_far":  # a dense lead (early copy) and the rest 1 GiB further on
        n = 30000
        lens = rng.integers(1000, 3000, n)
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
        offs[20000:] += 1 << 30
    elif shape == "shuffled_big":
        n = 50000
        lens = rng.integers(0, 9000, n)
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)[rng.permutation(n)]
    elif shape == "sparse_tail":
        n = 9000
        lens = rng.integers(0, 1500, n)
        offs = np.concatenate([[0], np.cumsum(lens + rng.integers(0, 1 << 20, n))[:-1]]).astype(np.int64) + 3
    elif shape == "zeros":
        n = 5000
        lens = np.zeros(n, np.int64)
        lens[::997] = 7
        offs = np.arange(n, dtype=np.int64) * 11 + 1
    elif shape == "one_byte_end":
        n = 4097
        lens = np.ones(n, np.int64)
        offs = np.arange(n, dtype=np.int64) * 2 + 15
    else:
        n = 200000
        lens = np.full(n, 1500)
        offs = np.arange(n, dtype=np.int64) * 1500
    arena_bytes = int((offs + lens).max()) + int(rng.integers(0, 5))
    segs = np.zeros(n, PESO_DTYPE)
    segs["offset"], segs["len"] = offs, lens
    chunk_knob(chunk_mb)
    check_plan(segs, arena_bytes)


def test_plan_refuses_a_segment_outside_the_arena():
    segs = np.zeros(3, PESO_DTYPE)
    segs["offset"], segs["len"] = [0, 100, 200], [100, 100, 101]
    bufs = np.zeros(2, np.uint64)
    rc = _lib.lib().tcsum_debug_plan_host_peso(segs.ctypes.data, 3, 300, None, 0, bufs.ctypes.data)
    assert rc == _lib.ERR_PARAM
