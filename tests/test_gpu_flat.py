"""k_flat_ipv4 -- the byte-window stream for IPv4 batches (plan + stream,
csum_device.h; libtcsum_bench.so's tcsum_flat_ipv4 since round 5, when it
left the product's route) -- against the reference's fixtures and the oracle (the CPU
restatement of net/src/tools.c:24-75 / pktbuf.c:646-670 and of the receive
gates of ipv4.c / tcp_in.c / udp.c / icmpv4.c, pinned to the reference's
own outputs).

Every workgroup sums a fixed byte window of the arena; packets that cross a
window boundary are combined from the windows' parts through one atomic word
per owner window, the last arriver finishing the packet.  The cases below put
packets, headers, checksum fields and packet ends on and across window
boundaries, make packets longer than several windows, crowd more packets into
one window than it has lanes, and break the stream precondition (descriptors
out of arena order, overlaps, a span the byte hint does not cover) so that
the per-packet fallback inside the same launch runs.  Bit-exact throughout.
"""
from devcopy import down, up
import numpy as np
import pytest

import golden_io as G

pytestmark = pytest.mark.gpu

WB = 12288  # the window: 4 waves x 64 lanes x 3 loads x 16 B (kFlatWB)


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "gpu tests need an MI355X"
    return t


@pytest.fixture(scope="module")
def prod(torch):
    from tcp_amd import build
    build.build()
    import tcp_amd
    tcp_amd.plat_init(0)
    return tcp_amd


class FlatStream:
    """The tcsum_batch_ipv4* calls the tests below make, run by the
    byte-window stream (libtcsum_bench.so's tcsum_flat_ipv4: round 5 took it
    out of libtcsum.so's route); every other attribute is tcp_amd's."""

    def __init__(self, tc, torch):
        self._tc, self._torch, self._split = tc, torch, 1

    def __getattr__(self, name):
        return getattr(self._tc, name)

    def debug_set(self, key, value):
        if key == "tx_split":  # the fill's two forms: stores in the kernel / deferred
            self._split = 1 if value == -1 else int(value)
        else:
            self._tc.debug_set(key, value)

    def _t(self, n, dt):
        return self._torch.empty(n, dtype=dt, device="cuda")

    def batch_ipv4(self, arena, d, n, total, out=None, flags=None, want_flags=True):
        out = self._t(n, self._torch.uint32) if out is None else out
        flags = self._t(n, self._torch.uint8) if flags is None and want_flags else flags
        self._tc.flat_ipv4(0, arena, d, n, total, out=out, flags=flags)
        return out, flags

    def batch_ipv4_rx_verify(self, arena, d, n, total, verdict=None, out=None, flags=None, want_flags=True):
        verdict = self._t(n, self._torch.int8) if verdict is None else verdict
        flags = self._t(n, self._torch.uint8) if flags is None and want_flags else flags
        self._tc.flat_ipv4(2, arena, d, n, total, out=out, flags=flags, verdict=verdict)
        return verdict, flags

    def batch_ipv4_tx_offload(self, arena, d, n, total, out=None, flags=None):
        out = self._t(n, self._torch.uint32) if out is None else out
        flags = self._t(n, self._torch.uint8) if flags is None else flags
        self._tc.flat_ipv4(3, arena, d, n, total, out=out, flags=flags)
        return out, flags

    def batch_ipv4_tx_fill(self, arena, d, n, total, out=None, flags=None, want_flags=True):
        flags = self._t(n, self._torch.uint8) if flags is None and want_flags else flags
        self._tc.flat_ipv4(4 if self._split else 1, arena, d, n, total, out=out, flags=flags)
        return flags


@pytest.fixture(scope="module")
def tc(prod, torch):
    return FlatStream(prod, torch)


def to_dev(torch, a: np.ndarray, pad: int = 256):
    t = torch.zeros(a.nbytes + pad, dtype=torch.uint8)
    t[: a.nbytes] = torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1))
    return up(t)


def _all_modes(tc, torch, oracle, host, pk, hint=None, tx=True):
    """sums, rx verify, tx offload and both tx fill forms vs the oracle
    (tx=False: overlapping packets, whose fill depends on the order)."""
    n = pk.size
    hint = int(pk["len"].astype(np.int64).sum()) if hint is None else hint
    arena = to_dev(torch, host)
    d = tc.descs_to_device(pk)
    out, fl = tc.batch_ipv4(arena, d, n, hint)
    exp, efl = oracle.batch_ipv4(host, pk, nthreads=8)
    np.testing.assert_array_equal(down(out), exp)
    np.testing.assert_array_equal(down(fl), efl)
    rout = torch.empty(n, dtype=torch.uint32, device="cuda")
    verdict, vfl = tc.batch_ipv4_rx_verify(arena, d, n, hint, out=rout)
    ev, evfl = oracle.batch_ipv4_rx_verify(host, pk, nthreads=8)
    np.testing.assert_array_equal(down(verdict), ev)
    np.testing.assert_array_equal(down(vfl), evfl)
    np.testing.assert_array_equal(down(rout), exp)  # rx reports the same sums
    if not tx:
        return
    tout, tfl = tc.batch_ipv4_tx_offload(arena, d, n, hint)
    filled = host.copy()
    tc.tx_apply_batch(filled, pk, down(tout), down(tfl))
    want = host.copy()
    oracle.batch_ipv4_tx_fill(want, pk, nthreads=8)
    np.testing.assert_array_equal(filled, want)
    for split in (0, 1):
        tc.debug_set("tx_split", split)
        a2 = to_dev(torch, host)
        fout = torch.empty(n, dtype=torch.uint32, device="cuda")
        tc.batch_ipv4_tx_fill(a2, d, n, hint, out=fout, want_flags=False)
        np.testing.assert_array_equal(down(a2)[: host.size], filled)
        np.testing.assert_array_equal(down(fout), down(tout))
    tc.debug_set("tx_split", -1)


def _headers(rng, host, offs, lens, valid=0.85):
    """Mostly plausible IPv4 headers (IHL 5..15, TCP/UDP/ICMP/other, stored
    checksums zero sometimes, fragments sometimes) over the random bytes."""
    for o, ln in zip(offs.tolist(), lens.tolist()):
        if ln < 20:
            continue
        h = host[o: o + 20]
        ihl = 5 if rng.random() < 0.8 else int(rng.integers(5, 16))
        h[0] = (0x40 | ihl) if rng.random() < valid else int(rng.integers(0, 256))
        tl = (ln if rng.random() < 0.8 else int(rng.integers(0, 70000))) & 0xFFFF  # a 16-bit field
        h[2], h[3] = tl >> 8, tl & 0xFF
        if rng.random() < 0.85:
            h[6], h[7] = 0, 0
        h[9] = int(rng.choice([6, 17, 1, 99]))
        if rng.random() < 0.2:
            h[10], h[11] = 0, 0
        hl = 4 * int(h[0] & 0xF)
        if ln >= hl + 20 and rng.random() < 0.2:
            host[o + hl + 16: o + hl + 18] = 0
            host[o + hl + 6: o + hl + 8] = 0


def _arena(rng, size):
    host = rng.integers(0, 256, size, dtype=np.uint8)
    for _ in range(30):  # runs of 0x00 / 0xFF: fold edge cases
        a = int(rng.integers(0, max(1, size - 5000)))
        host[a: a + int(rng.integers(1, 5000))] = rng.choice([0, 0xFF])
    return host


def _stream(lens, start=0, gaps=None):
    step = lens + (0 if gaps is None else gaps)
    return start + np.concatenate([[0], np.cumsum(step[:-1])]).astype(np.int64)


def _pk(tc, offs, lens):
    pk = np.zeros(len(lens), tc.PKT_DTYPE)
    pk["offset"], pk["len"] = offs, lens
    return pk


@pytest.mark.parametrize("seed", range(10))
def test_flat_fuzz_vs_oracle(tc, torch, oracle, seed):
    """Packets of 0..9000 B (a third of them short), packed or with gaps, at a
    random arena phase; every mode and both fill forms."""
    rng = np.random.default_rng(7700 + seed)
    n = int(rng.integers(500, 5000))
    kind = rng.integers(0, 3, n)
    lens = np.where(kind == 0, rng.integers(0, 80, n),
                    np.where(kind == 1, rng.integers(20, 2048, n), rng.integers(20, 9001, n)))
    gaps = rng.integers(0, 40, n) * (rng.random(n) < 0.3) if seed % 2 else None
    offs = _stream(lens, int(rng.integers(0, 200)), gaps)
    host = _arena(rng, int(offs[-1] + lens[-1]) + 512)
    _headers(rng, host, offs, lens)
    _all_modes(tc, torch, oracle, host, _pk(tc, offs, lens))


@pytest.mark.parametrize("phase", [0, 1, 5, 10, 11, 12, 15, 16, 18, 19, 20, 35, 36, 37, 77, 78])
def test_flat_boundaries(tc, torch, oracle, phase):
    """A packet placed so that its header, its IPv4 checksum field, its L4
    checksum field or its end lands on / across every window boundary, at
    every offset near it: 2,000 packets of 700..1400 B laid out so that one
    of them starts `phase` bytes before each boundary."""
    rng = np.random.default_rng(phase)

    def fill(total):  # packets of 700..1400 B that add up to `total` exactly
        out = []
        while total > 2100:
            out.append(int(rng.integers(700, 1401)))
            total -= out[-1]
        if total <= 1400:
            out.append(total)
        else:
            out += [total // 2, total - total // 2]
        return out

    # window boundaries sit at k * WB (the arena starts on a 128-B line): the
    # first packet of every stretch starts `phase` bytes before a boundary
    lens = fill(WB - phase)
    while len(lens) < 2000:
        lens += fill(WB)
    lens = np.array(lens, np.int64)
    offs = _stream(lens)
    host = _arena(rng, int(offs[-1] + lens[-1]) + 512)
    _headers(rng, host, offs, lens, valid=0.95)
    _all_modes(tc, torch, oracle, host, _pk(tc, offs, lens))


def test_flat_long_packets(tc, torch, oracle):
    """Packets longer than one window and up to the IPv4 maximum (65,535 B)
    -- spread over up to seven windows, their parts combined by the last
    arriving one -- among short ones; frames longer than the IPv4 maximum."""
    rng = np.random.default_rng(99)
    n = 400
    lens = np.where(rng.random(n) < 0.3, rng.integers(12000, 65536, n), rng.integers(20, 3000, n)).astype(np.int64)
    lens[[5, 77]] = [70000, 131072]  # frames past total_len's range: loads stop at 65,600 B
    offs = _stream(lens, 3)
    host = _arena(rng, int(offs[-1] + lens[-1]) + 512)
    _headers(rng, host, offs, lens, valid=0.95)
    _all_modes(tc, torch, oracle, host, _pk(tc, offs, lens))


def test_flat_crowded_windows(tc, torch, oracle):
    """20..64-B packets: more packets start in one 12-KiB window than it has
    lanes (256), so the window takes several rounds of them; and runs of
    frames shorter than 20 B (SHORT) across boundaries."""
    rng = np.random.default_rng(5)
    n = 60000
    lens = np.where(rng.random(n) < 0.1, rng.integers(0, 20, n), rng.integers(20, 65, n)).astype(np.int64)
    offs = _stream(lens, 9)
    host = _arena(rng, int(offs[-1] + lens[-1]) + 512)
    _headers(rng, host, offs, lens)
    _all_modes(tc, torch, oracle, host, _pk(tc, offs, lens))


@pytest.mark.parametrize("layout", ["shuffled", "overlap", "reversed", "big_gaps", "tiny_hint"])
def test_flat_not_a_stream_falls_back(tc, torch, oracle, layout):
    """Batches the stream cannot take -- descriptors out of arena order,
    overlapping packets, gaps the byte hint does not cover -- are found by the
    plan and summed packet by packet in the same launch: still exact."""
    rng = np.random.default_rng(["shuffled", "overlap", "reversed", "big_gaps", "tiny_hint"].index(layout))
    n = 3000
    lens = rng.integers(20, 9001, n).astype(np.int64)
    offs = _stream(lens, 1, rng.integers(0, 2000, n) if layout == "big_gaps" else None)
    if layout == "overlap":
        offs[100:] -= 30
    host = _arena(rng, int(offs.max() + lens.max()) + 512)
    _headers(rng, host, offs, lens)
    pk = _pk(tc, offs, lens)
    if layout == "shuffled":
        pk = pk[rng.permutation(n)]
    elif layout == "reversed":
        pk = pk[::-1].copy()
    hint = int(lens.sum()) // 4 if layout == "tiny_hint" else None
    _all_modes(tc, torch, oracle, host, pk, hint=hint, tx=layout != "overlap")


@pytest.mark.parametrize("fixture", ["ipv4", "rx", "tx", "stack_tx"])
def test_flat_reference_fixtures(tc, torch, fixture):
    """The reference's own outputs (tests/golden) through the stream path."""
    if fixture == "ipv4":
        cases, pool = G.ipv4_cases()
        pk = np.zeros(cases.size, tc.PKT_DTYPE)
        pk["offset"], pk["len"] = cases["pool_off"], cases["frame_len"]
        out, flags = tc.batch_ipv4(to_dev(torch, pool), tc.descs_to_device(pk), pk.size, int(pk["len"].sum()))
        out = down(out)
        np.testing.assert_array_equal(out & 0xFFFF, cases["ip"])
        np.testing.assert_array_equal(out >> 16, cases["l4"])
        np.testing.assert_array_equal(down(flags), cases["flags"])
    elif fixture == "rx":
        cases, pool = G.ipv4_rx_cases()
        pk = G.pkt_descs(cases, tc.PKT_DTYPE)
        verdict, flags = tc.batch_ipv4_rx_verify(to_dev(torch, pool), tc.descs_to_device(pk), cases.size,
                                                 int(pk["len"].sum()))
        np.testing.assert_array_equal(down(verdict), cases["verdict"])
        np.testing.assert_array_equal(down(flags), cases["flags"])
    else:
        cases, pin, pout = G.ipv4_tx_cases() if fixture == "tx" else G.stack_tx_cases()
        pk = G.pkt_descs(cases, tc.PKT_DTYPE)
        for split in (0, 1):
            tc.debug_set("tx_split", split)
            arena = to_dev(torch, pin)
            flags = tc.batch_ipv4_tx_fill(arena, tc.descs_to_device(pk), cases.size, int(pk["len"].sum()))
            np.testing.assert_array_equal(down(arena)[: pout.size], pout)
            np.testing.assert_array_equal(down(flags), cases["flags"])


@pytest.mark.parametrize("config", ["mixed", "mixed_aligned"])
def test_flat_full_mixed_config(tc, torch, oracle, config):
    """configs[3] at full size (1M packets, 4.4 GiB) through the stream:
    both sums of every packet equal the oracle's; then fill, verify (all
    OK), corrupt 2,000 packets, verify again against the oracle."""
    from tcp_amd import workload
    b = workload.make_batch(config)
    arena, descs = workload.materialize(b)
    out, fl = tc.batch_ipv4(arena, descs, b.n, b.total_bytes)
    host = down(arena)
    exp, efl = oracle.batch_ipv4(host, b.descs, nthreads=16)
    np.testing.assert_array_equal(down(out), exp)
    np.testing.assert_array_equal(down(fl), efl)
    del host
    tc.batch_ipv4_tx_fill(arena, descs, b.n, b.total_bytes)
    verdict, _ = tc.batch_ipv4_rx_verify(arena, descs, b.n, b.total_bytes)
    assert (down(verdict) == 0).all()
    rng = np.random.default_rng(55)
    bad = rng.choice(b.n, 2000, replace=False)
    pos = (b.descs["offset"][bad] + 20 + (rng.integers(0, 1 << 30, bad.size) % (b.descs["len"][bad] - 20)))
    arena[up(torch.from_numpy(pos.astype(np.int64)))] ^= 0x04
    verdict, flags = tc.batch_ipv4_rx_verify(arena, descs, b.n, b.total_bytes)
    v = down(verdict)
    ev, ef = oracle.batch_ipv4_rx_verify(down(arena), b.descs, nthreads=16)
    np.testing.assert_array_equal(v, ev)
    np.testing.assert_array_equal(down(flags), ef)
    assert (v[bad] == -13).mean() > 0.99


@pytest.mark.parametrize("layout", ["packed", "shuffled"])
def test_ipv4_layout_hints_give_the_same_results(prod, torch, oracle, layout):
    """tcsum_batch's layout hint on every IPv4 operation (sums, rx verify, tx
    offload, tx fill) changes only the kernel, never a result -- also when an
    ORDERED promise is false (a shuffled batch)."""
    tc = prod
    rng = np.random.default_rng(300 + (layout == "shuffled"))
    lens = rng.integers(20, 9000, 3000).astype(np.int64)
    offs = _stream(lens, 7)
    host = _arena(rng, int(offs[-1] + lens[-1]) + 512)
    _headers(rng, host, offs, lens, valid=0.9)
    pk = _pk(tc, offs, lens)
    if layout == "shuffled":
        pk = pk[rng.permutation(pk.size)]
    n, total = pk.size, int(lens.sum())
    exp, efl = oracle.batch_ipv4(host, pk, nthreads=8)
    ev, evfl = oracle.batch_ipv4_rx_verify(host, pk, nthreads=8)
    want = host.copy()
    oracle.batch_ipv4_tx_fill(want, pk, nthreads=8)
    d = tc.descs_to_device(pk)
    for lay in (tc.LAYOUT_UNKNOWN, tc.LAYOUT_ORDERED, tc.LAYOUT_SHUFFLED):
        arena = to_dev(torch, host)
        fl = torch.empty(n, dtype=torch.uint8, device="cuda")
        out, _, _ = tc.batch(tc.OP_IPV4, arena, d, n, flags=fl, total_bytes=total, layout=lay)
        np.testing.assert_array_equal(down(out), exp)
        np.testing.assert_array_equal(down(fl), efl)
        rout = torch.empty(n, dtype=torch.uint32, device="cuda")
        _, _, v = tc.batch(tc.OP_IPV4_RX_VERIFY, arena, d, n, out=rout, total_bytes=total, layout=lay)
        np.testing.assert_array_equal(down(v), ev)
        np.testing.assert_array_equal(down(rout), exp)
        tout, tfl, _ = tc.batch(tc.OP_IPV4_TX_OFFLOAD, arena, d, n, total_bytes=total, layout=lay)
        filled = host.copy()
        tc.tx_apply_batch(filled, pk, down(tout), down(tfl))
        np.testing.assert_array_equal(filled, want)
        tc.batch(tc.OP_IPV4_TX_FILL, arena, d, n, total_bytes=total, layout=lay)
        np.testing.assert_array_equal(down(arena)[: host.size], want)
