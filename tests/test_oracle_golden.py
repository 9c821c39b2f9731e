"""Pin the CPU oracle to the reference's own outputs (tests/golden/).

Every expected value in the fixtures is what the reference's checksum16 /
pktbuf_checksum16 / checksum_peso returned (net/src/tools.c:24-75,
net/src/pktbuf.c:646-670), compiled from /root/reference by oracle/golden_gen.c.
"""
import numpy as np
import pytest

import golden_io as G


def test_kats(oracle):
    k = G.kat_inputs()
    h, e = k["KAT-1"]
    assert oracle.checksum16(0, h, 20, 0, 1) == e == 0x61B8
    filled = bytearray(h)
    filled[10:12] = e.to_bytes(2, "little")
    assert oracle.checksum16(0, filled, 20, 0, 1) == 0
    b, e = k["KAT-2"]
    assert oracle.flat_checksum16(b, 0, 1) == e == 0x8EE9
    assert oracle.checksum16(0, b, 999, 0, 1) == e
    b, e = k["KAT-3"]
    assert oracle.checksum_peso(b, bytes([192, 168, 74, 3]), bytes([192, 168, 74, 2]), 6) == e == 0x4AD0
    b, e = k["KAT-4"]
    assert oracle.checksum16(0, b, 4, 0, 1) == e == 0xFFFF
    b, e = k["KAT-5"]
    assert oracle.checksum16(0, b, 2, 0, 1) == e == 0x0000


def test_flat_checksum16(oracle):
    pool = G.pool()
    cases = G.flat_cases()
    assert cases.size == 6000
    bad = []
    for c in cases:
        off, n = int(c["pool_off"]), int(c["len"])
        got = oracle.checksum16(int(c["offset"]), pool[off: off + n], n, int(c["pre_sum"]),
                                int(c["complement"]))
        if got != int(c["expected"]):
            bad.append((c, got))
    assert not bad, bad[:5]


def test_pktbuf_checksum16(oracle):
    pool = G.pool()
    cases, blocks = G.pktbuf_cases()
    assert cases.size == 1500
    for c in cases:
        pieces = G.case_blocks(c, blocks, pool)
        # drop the bytes before the cursor (pktbuf_seek), keeping block shapes
        skip, rest = int(c["seek"]), []
        for p in pieces:
            if skip >= p.size:
                skip -= p.size
                continue
            rest.append(p[skip:])
            skip = 0
        got = oracle.pieces_checksum16(rest, int(c["len"]), int(c["pre_sum"]), int(c["complement"]))
        assert got == int(c["expected"]), c


def test_checksum_peso(oracle):
    pool = G.pool()
    cases, _ = G.peso_cases()
    assert cases.size == 1248
    for c in cases:
        off, n = int(c["pool_off"]), int(c["total"])
        got = oracle.checksum_peso(pool[off: off + n], c["dst"], c["src"], int(c["proto"]))
        assert got == int(c["expected"]), c


def test_ipv4_pair(oracle):
    cases, ipool = G.ipv4_cases()
    assert cases.size == 500
    for c in cases:
        off, n = int(c["pool_off"]), int(c["frame_len"])
        ip, l4, fl = oracle.ipv4_pair(ipool[off: off + max(n, 1)], n)
        assert (ip, l4, fl) == (int(c["ip"]), int(c["l4"]), int(c["flags"])), c


def test_ipv4_tx_fill(oracle):
    cases, pin, pout = G.ipv4_tx_cases()
    assert cases.size == 400
    arena = pin.copy()
    flags = oracle.batch_ipv4_tx_fill(arena, G.pkt_descs(cases, oracle.PKT_DTYPE), nthreads=4)
    np.testing.assert_array_equal(flags, cases["flags"])
    np.testing.assert_array_equal(arena, pout)
    assert (pin != pout).any()


def test_stack_tx_fill(oracle):
    """The reference stack's own transmitted frames (udp_out, send_out,
    icmpv4_out, ipv4_out, ip_frag_out): the fill restores every byte."""
    cases, pin, pout = G.stack_tx_cases()
    assert cases.size > 1000
    arena = pin.copy()
    flags = oracle.batch_ipv4_tx_fill(arena, G.pkt_descs(cases, oracle.PKT_DTYPE), nthreads=4)
    np.testing.assert_array_equal(flags, cases["flags"])
    np.testing.assert_array_equal(arena, pout)
    kinds = cases["kind"]
    for proto in (1, 6, 17):
        assert ((kinds >> 8) == proto).sum() >= 100, proto
    assert (kinds & 1).sum() >= 100  # fragments: header checksum only
    assert ((kinds >> 8) > 17).sum() >= 20  # other protocols (raw)


def test_ipv4_rx_verify(oracle):
    """Verdicts of the reference stack's receive path (oracle/stack_gen.c)."""
    cases, pool = G.ipv4_rx_cases()
    assert cases.size > 4000
    verdict, flags = oracle.batch_ipv4_rx_verify(pool, G.pkt_descs(cases, oracle.PKT_DTYPE), nthreads=4)
    np.testing.assert_array_equal(verdict, cases["verdict"])
    np.testing.assert_array_equal(flags, cases["flags"])
    # the fixture reaches every gate of every receive function
    gate, proto, v = cases["gate"] & 0xFF, cases["gate"] >> 8, cases["verdict"]
    for g, p, code, at_least in [(1, None, -5, 20), (1, None, -11, 20), (1, None, -13, 20),
                                 (2, None, 0, 100), (3, 6, 0, 100), (3, 6, -1, 10), (3, 6, -13, 50),
                                 (3, 6, -5, 5), (3, 17, 0, 100), (3, 17, -5, 10), (3, 17, -13, 50),
                                 (3, 17, -14, 20), (3, 1, 0, 50), (3, 1, -5, 10)]:
        sel = (gate == g) & (v == code) & ((proto == p) if p is not None else True)
        assert sel.sum() >= at_least, (g, p, code, int(sel.sum()))
    assert ((gate == 3) & (proto != 1) & (proto != 6) & (proto != 17)).sum() >= 20  # raw_in


def test_ipv4_rx_tcp_gates_behind_checksum(oracle):
    """tcp_in.c:87-103: with a valid checksum, the data-offset, port and flag
    gates decide -- each reached by the reference-stack fixture."""
    cases, pool = G.ipv4_rx_cases()
    pk = G.pkt_descs(cases, oracle.PKT_DTYPE)
    out, _ = oracle.batch_ipv4(pool, pk, nthreads=4)
    seen = {"doff": 0, "port": 0, "flag": 0}
    for i in np.nonzero(((cases["gate"] & 0xFF) == 3) & ((cases["gate"] >> 8) == 6))[0]:
        o = int(cases["pool_off"][i])
        ihl = int(pool[o] & 15) * 4
        t = pool[o + ihl: o + ihl + 20]
        if (t[16] | t[17]) and (out[i] >> 16):
            continue  # the checksum gate decided
        v = int(cases["verdict"][i])
        if v == -5:
            seen["doff"] += 1
        elif v == -13 and (not (t[0] | t[1]) or not (t[2] | t[3])):
            seen["port"] += 1
        elif v == -13:
            assert not (t[12] | t[13])
            seen["flag"] += 1
    assert min(seen.values()) >= 5, seen


def test_batch_forms_agree_with_scalar(oracle):
    """The threaded batch entry points are the scalar routines, per item."""
    pool = G.pool()
    cases, _ = G.peso_cases()
    segs = np.zeros(cases.size, oracle.PESO_DTYPE)
    segs["offset"] = cases["pool_off"]
    segs["len"] = cases["total"]
    segs["src"] = cases["src"]
    segs["dst"] = cases["dst"]
    segs["protocol"] = cases["proto"]
    out = oracle.batch_peso(pool, segs, nthreads=4)
    np.testing.assert_array_equal(out, cases["expected"].astype(np.uint16))

    icases, ipool = G.ipv4_cases()
    pk = np.zeros(icases.size, oracle.PKT_DTYPE)
    pk["offset"] = icases["pool_off"]
    pk["len"] = icases["frame_len"]
    out, flags = oracle.batch_ipv4(ipool, pk, nthreads=3)
    np.testing.assert_array_equal(out & 0xFFFF, icases["ip"])
    np.testing.assert_array_equal(out >> 16, icases["l4"])
    np.testing.assert_array_equal(flags, icases["flags"])


@pytest.mark.parametrize("n", [0, 1, 2, 127, 128, 1500, 65535, 65536, 65537, 200000])
def test_closed_form(oracle, n):
    """S = pre + sum b[i]*256^(i&1); fold(S) = 0 if S == 0 else 1 + (S-1) % 0xFFFF."""
    rng = np.random.default_rng(n)
    b = rng.integers(0, 256, n, dtype=np.uint8)
    pre = int(rng.integers(0, 0x10000))
    s = pre + int(b[0::2].astype(np.uint64).sum()) + 256 * int(b[1::2].astype(np.uint64).sum())
    f = 0 if s == 0 else 1 + (s - 1) % 0xFFFF
    assert oracle.flat_checksum16(b, pre, 0) == f
    assert oracle.flat_checksum16(b, pre, 1) == (~f) & 0xFFFF


def test_synth_fill_is_splitmix(oracle):
    a = oracle.synth_fill(0, 64, 7)
    b = oracle.synth_fill(13, 40, 7)
    np.testing.assert_array_equal(a[13:53], b)
