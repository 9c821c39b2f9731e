"""k_segments_pk's descriptor prefetch on its range-by-range path (debug
knob "pf_dist", csum_device.h prefetch_descs: lanes of wave 0 touch the
descriptor lines of the workgroup pf_dist logical blocks ahead).  It may not
change a result or read past the descriptor array: both
descriptor layouts (checksum_peso, pktbuf_checksum16) against the oracle,
packed, shuffled, TSO-sized and K = 8 batches, distances from 1 to far past
the grid, descriptor arrays at the end of their allocation; and the IPv4
kernels, which must be unaffected by the knob."""
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
    t.copy_(torch.from_numpy(raw.copy()))
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
    arena = torch.from_numpy(host).cuda()
    d = _descs_at_end(torch, tc, p)
    with tc.debug(pf_dist=pf):
        got = tc.batch_peso(arena, d, n, int(lens.sum())).cpu().numpy()
        segs = np.zeros(n, tc.SEG_DTYPE)  # the same ranges as pktbuf_checksum16 (16-B descriptors)
        segs["offset"], segs["len"], segs["pre_sum"] = p["offset"], p["len"], rng.integers(0, 1 << 17, n)
        gs = tc.batch_segments(arena, _descs_at_end(torch, tc, segs), n, 1, int(lens.sum())).cpu().numpy()
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(gs, oracle.batch_segments(host, segs, 1, nthreads=8))
    # the per-range kernels (the SHUFFLED route) with their own prefetch knob
    with tc.debug(pf_range=pf):
        gr, _, _ = tc.batch(tc.OP_PESO, arena, d, n, total_bytes=int(lens.sum()), layout=tc.LAYOUT_SHUFFLED)
    np.testing.assert_array_equal(gr.cpu().numpy(), want)


@pytest.mark.parametrize("pf", DISTANCES)
def test_ipv4_batches_with_prefetch(tc, torch, oracle, pf):
    from tcp_amd import workload
    b = workload.make_batch("mixed", n=9001)
    arena, descs = workload.materialize(b)
    host = arena.cpu().numpy()
    d = _descs_at_end(torch, tc, b.descs)
    eo, ef = oracle.batch_ipv4(host, b.descs, nthreads=8)
    ev, _ = oracle.batch_ipv4_rx_verify(host, b.descs, nthreads=8)
    want = host.copy()
    oracle.batch_ipv4_tx_fill(want, b.descs, nthreads=8)
    with tc.debug(pf_dist=pf):
        out, fl = tc.batch_ipv4(arena, d, b.n, b.total_bytes)
        v, _ = tc.batch_ipv4_rx_verify(arena, d, b.n, b.total_bytes)
        for split in (0, 1):
            a2 = arena.clone()
            with tc.debug(tx_split=split):
                tc.batch_ipv4_tx_fill(a2, d, b.n, b.total_bytes)
            np.testing.assert_array_equal(a2.cpu().numpy(), want)
    np.testing.assert_array_equal(out.cpu().numpy(), eo)
    np.testing.assert_array_equal(fl.cpu().numpy(), ef)
    np.testing.assert_array_equal(v.cpu().numpy(), ev)
