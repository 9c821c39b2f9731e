"""k_segments_pk's descriptor prefetch on its range-by-range path (debug
knob "pf_dist", csum_device.h prefetch_descs: lanes of wave 0 touch the
descriptor lines of the workgroup pf_dist logical blocks ahead).  It may not
change a result or read past the descriptor array: both
descriptor layouts (checksum_peso, pktbuf_checksum16) against the oracle,
packed, shuffled, TSO-sized and K = 8 batches, distances from 1 to far past
the grid, descriptor arrays at the end of their allocation; and the IPv4
kernels, which must be unaffected by the knob.  Also the same path's scalar
descriptor reads (debug knob "pk_early") for every group width."""
from devcopy import down, up
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

DISTANCES = [0, 1, 7, 512, 2048, 1 << 22]


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "gpu tests need an MI355X"
    return t


@pytest.fixture(scope="module")
def tc(torch):
    from tcp_amd import build
    build.build()
    import tcp_amd
    tcp_amd.plat_init(0)
    return tcp_amd


def _descs_at_end(torch, tc, descs):
    """The descriptor bytes at the very end of their own allocation: a read
    past the array would leave it (and the allocator's page)."""
    raw = np.ascontiguousarray(descs).view(np.uint8)
    t = torch.empty(raw.size, dtype=torch.uint8, device="cuda")
    t.copy_(torch.from_numpy(raw.copy()).pin_memory())
    return t


@pytest.mark.parametrize("pf", DISTANCES)
@pytest.mark.parametrize("layout", ["packed", "shuffled", "tso", "mtu"])
def test_peso_batches_with_prefetch(tc, torch, oracle, pf, layout):
    rng = np.random.default_rng(40 + DISTANCES.index(pf))
    if layout == "tso":
        n, lens = 300, np.full(300, 65536)
    elif layout == "mtu":  # K = 8 full workgroups, the last one partial
        n, lens = 8 * 1001 + 5, np.full(8 * 1001 + 5, 1500)
    else:
        n = 20011
        lens = rng.integers(0, 3001, n)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64) + 3
    host = rng.integers(0, 256, int(offs[-1] + lens[-1]) + 64, dtype=np.uint8)
    p = np.zeros(n, tc.PESO_DTYPE)
    p["offset"], p["len"] = offs, lens
    p["src"] = rng.integers(0, 256, (n, 4))
    p["dst"] = rng.integers(0, 256, (n, 4))
    p["protocol"] = rng.choice([6, 17], n)
    if layout == "shuffled":
        p = p[rng.permutation(n)]
    want = oracle.batch_peso(host, p, nthreads=8)
    arena = up(torch.from_numpy(host))
    d = _descs_at_end(torch, tc, p)
    with tc.debug(pf_dist=pf):
        got = down(tc.batch_peso(arena, d, n, int(lens.sum())))
        segs = np.zeros(n, tc.SEG_DTYPE)  # the same ranges as pktbuf_checksum16 (16-B descriptors)
        segs["offset"], segs["len"], segs["pre_sum"] = p["offset"], p["len"], rng.integers(0, 1 << 17, n)
        gs = down(tc.batch_segments(arena, _descs_at_end(torch, tc, segs), n, 1, int(lens.sum())))
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(gs, oracle.batch_segments(host, segs, 1, nthreads=8))
    # the per-range kernels (the SHUFFLED route for short ranges) with their own prefetch knob
    with tc.debug(pf_range=pf, packed=0):
        gr, _, _ = tc.batch(tc.OP_PESO, arena, d, n, total_bytes=int(lens.sum()), layout=tc.LAYOUT_SHUFFLED)
    np.testing.assert_array_equal(down(gr), want)


@pytest.mark.parametrize("pf", DISTANCES)
def test_ipv4_batches_with_prefetch(tc, torch, oracle, pf):
    from tcp_amd import workload
    b = workload.make_batch("mixed", n=9001)
    arena, descs = workload.materialize(b)
    host = down(arena)
    d = _descs_at_end(torch, tc, b.descs)
    eo, ef = oracle.batch_ipv4(host, b.descs, nthreads=8)
    ev, _ = oracle.batch_ipv4_rx_verify(host, b.descs, nthreads=8)
    want = host.copy()
    oracle.batch_ipv4_tx_fill(want, b.descs, nthreads=8)
    with tc.debug(pf_dist=pf):
        out, fl = tc.batch_ipv4(arena, d, b.n, b.total_bytes)
        v, _ = tc.batch_ipv4_rx_verify(arena, d, b.n, b.total_bytes)
        for split, warm in ((0, None), (1, None), (1, 0)):
            a2 = arena.clone()
            with tc.debug(tx_split=split, tx_warm=warm):
                tc.batch_ipv4_tx_fill(a2, d, b.n, b.total_bytes)
            np.testing.assert_array_equal(down(a2), want)
    np.testing.assert_array_equal(down(out), eo)
    np.testing.assert_array_equal(down(fl), ef)
    np.testing.assert_array_equal(down(v), ev)


EARLY_LAYOUTS = ["packed", "shuffled", "mtu", "wide", "tail", "mid", "small", "tiny", "k17", "s400",
                 "s200", "tinyp", "tinyswap"]


@pytest.mark.parametrize("early", [1, 0])
@pytest.mark.parametrize("layout", EARLY_LAYOUTS)
def test_pk_early_descriptors(tc, torch, oracle, layout, early):
    """debug "pk_early" (default 1): a packed-kernel workgroup on its
    range-by-range path (K <= 32) reads its ranges' descriptors with scalar
    loads, each lane group picking its own (0: vector loads; K > 32 always
    vector loads, one per round of ranges).  Both descriptor layouts, a last
    workgroup with fewer ranges (tail), K = 3 (wide: 64-lane groups), 8 (32),
    ~12 (mid: 16), ~21 (small) and 17 (k17: 16 lanes, a second round for the
    last ranges), ~30 (s400: 8 lanes x 4 loads), ~61 (s200: 8 lanes, two
    rounds), ~190 (tiny: 4 lanes, three rounds; tinyp: packed, the region
    path; tinyswap: packed with middle ranges swapped between workgroups 100
    apart, so the span holds and the region check fails), shuffled and
    packed, against the oracle; the descriptors end their allocation."""
    rng = np.random.default_rng(77 + EARLY_LAYOUTS.index(layout))
    if layout == "mid":
        n, lens = 15013, rng.integers(800, 1200, 15013)
    elif layout == "small":
        n, lens = 30011, np.full(30011, 576)
    elif layout in ("tiny", "tinyp", "tinyswap"):
        n, lens = 60013, rng.integers(1, 128, 60013)
    elif layout == "s200":
        n, lens = 40009, rng.integers(150, 250, 40009)
    elif layout == "k17":
        n, lens = 17 * 1003 + 9, rng.integers(650, 790, 17 * 1003 + 9)
    elif layout == "s400":
        n, lens = 40009, rng.integers(300, 500, 40009)
    elif layout == "mtu":
        n, lens = 8 * 1001, np.full(8 * 1001, 1500)
    elif layout == "wide":  # ~4 KiB ranges: K = 3, one 64-lane group per range
        n, lens = 3001, rng.integers(3500, 4500, 3001)
    elif layout == "tail":
        n, lens = 8 * 997 + 3, np.full(8 * 997 + 3, 1500)
    else:
        n = 20011
        lens = rng.integers(1000, 2000, n)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64) + 5
    host = rng.integers(0, 256, int(offs[-1] + lens[-1]) + 64, dtype=np.uint8)
    p = np.zeros(n, tc.PESO_DTYPE)
    p["offset"], p["len"] = offs, lens
    p["src"] = rng.integers(0, 256, (n, 4))
    p["dst"] = rng.integers(0, 256, (n, 4))
    p["protocol"] = rng.choice([6, 17], n)
    if layout in ("shuffled", "wide", "tail", "mid", "small", "tiny", "k17", "s400", "s200"):
        p = p[rng.permutation(n)]
    elif layout == "tinyswap":
        K = tc.route(int(lens.mean()))["packed"]
        assert K > 32
        for k in range(0, n // K - 100, 7):
            i, j = K * k + K // 2, K * (k + 100) + K // 3
            p[[i, j]] = p[[j, i]]
    want = oracle.batch_peso(host, p, nthreads=8)
    arena = up(torch.from_numpy(host))
    segs = np.zeros(n, tc.SEG_DTYPE)
    segs["offset"], segs["len"], segs["pre_sum"] = p["offset"], p["len"], rng.integers(0, 1 << 17, n)
    with tc.debug(pk_early=early, packed=1):
        got = down(tc.batch_peso(arena, _descs_at_end(torch, tc, p), n, int(lens.sum())))
        gs = down(tc.batch_segments(arena, _descs_at_end(torch, tc, segs), n, 1, int(lens.sum())))
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(gs, oracle.batch_segments(host, segs, 1, nthreads=8))


@pytest.mark.parametrize("sdesc", [1, 0])
@pytest.mark.parametrize("shape", [(8, 4), (16, 3), (16, 4), (16, 6), (16, 8), (32, 6), (4, 2)])
def test_per_range_scalar_descriptors(tc, torch, oracle, shape, sdesc):
    """debug "seg_sdesc" (default 1): the per-range kernel with 8 or 16 lanes
    per range reads its wave's descriptors with scalar loads, each lane group
    picking its own; other widths keep their vector loads.  Every forced
    shape, both descriptor layouts, a last workgroup with fewer ranges and the
    descriptor array at the end of its allocation, shuffled, against the
    oracle."""
    g, u = shape
    rng = np.random.default_rng(500 + 10 * g + u + sdesc)
    n = 7 * (256 // g) + 3  # a short last workgroup
    lens = rng.integers(0, 1200, n)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64) + 1
    host = rng.integers(0, 256, int(offs[-1] + lens[-1]) + 64, dtype=np.uint8)
    p = np.zeros(n, tc.PESO_DTYPE)
    p["offset"], p["len"] = offs, lens
    p["src"] = rng.integers(0, 256, (n, 4))
    p["dst"] = rng.integers(0, 256, (n, 4))
    p["protocol"] = rng.choice([6, 17], n)
    p = p[rng.permutation(n)]
    segs = np.zeros(n, tc.SEG_DTYPE)
    segs["offset"], segs["len"], segs["pre_sum"] = p["offset"], p["len"], rng.integers(0, 1 << 17, n)
    arena = up(torch.from_numpy(host))
    with tc.debug(seg_sdesc=sdesc, packed=0, lanes=g, loads=u):
        got = down(tc.batch_peso(arena, _descs_at_end(torch, tc, p), n, int(lens.sum())))
        gs = down(tc.batch_segments(arena, _descs_at_end(torch, tc, segs), n, 1, int(lens.sum())))
    np.testing.assert_array_equal(got, oracle.batch_peso(host, p, nthreads=8))
    np.testing.assert_array_equal(gs, oracle.batch_segments(host, segs, 1, nthreads=8))
