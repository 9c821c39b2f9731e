"""Capture files on the rx path (tcsum_pcap_index, tcp_amd.pcap).

CPU: the index over savefiles written by tests/pcap_build.py (every link
type, byte order and timestamp unit; FCS; truncated records and files) against
the offsets the writer recorded, and the rx front end's per-frame decision
(plat/netif_pcap.c:9-38, net/src/ether.c:14-25,62-101).
GPU: the reference's own rx fixtures (tests/golden/ipv4_rx_*.bin, verdicts
from the compiled reference stack) wrapped into captures and verified in
place through tcsum_host_batch_ipv4_rx_verify.
"""
from devcopy import down
import numpy as np
import pytest

import golden_io as G
import pcap_build as PB

OK, SIZE, NOT_SUPPORT, PARAM, MEM, ARP = 0, -5, -11, -7, -2, 1


def golden_frames():
    cases, pool = G.ipv4_rx_cases()
    frames = [pool[o: o + n].tobytes() for o, n in zip(cases["pool_off"], cases["frame_len"])]
    return cases, frames


@pytest.fixture(scope="module")
def pcap():
    from tcp_amd import pcap
    return pcap


@pytest.mark.parametrize("big_endian", [False, True])
@pytest.mark.parametrize("nanosecond", [False, True])
@pytest.mark.parametrize("link", [PB.ETHER, PB.RAW, PB.IPV4, PB.NULL, PB.SLL])
def test_index_offsets(pcap, link, big_endian, nanosecond):
    cases, frames = golden_frames()
    frames = [f for f in frames if len(f) <= 1500]  # ether's is_pkt_ok bound for every link type here
    buf, offs, lens = PB.build(frames, link, big_endian, nanosecond)
    pkts, l2 = pcap.index(buf)
    assert pkts.size == len(frames)
    ipv4 = np.ones(len(frames), bool)  # raw links: every frame goes to ipv4_in, whose gates judge it
    np.testing.assert_array_equal(l2[ipv4], OK)
    np.testing.assert_array_equal(l2[~ipv4], NOT_SUPPORT)
    np.testing.assert_array_equal(pkts["offset"][ipv4], offs[ipv4])
    np.testing.assert_array_equal(pkts["len"][ipv4], lens[ipv4])
    assert (pkts["len"][~ipv4] == 0).all()
    for i in np.flatnonzero(ipv4)[:50]:  # the descriptor addresses the frame's own bytes
        o, n = int(pkts["offset"][i]), int(pkts["len"][i])
        assert buf[o: o + n] == frames[i]


def test_ether_front_end_decisions(pcap):
    """ether_in: is_pkt_ok size bounds (14..1514), ARP to arp_in, other types
    NOT_SUPPORT (ether.c:14-25,75-97); an FCS the file declares is not L3."""
    body = bytes(range(40))
    frames = [body, body, body, b"", bytes(1500), bytes(1501), body]
    types = [0x0800, 0x0806, 0x86DD, 0x0800, 0x0800, 0x0800, 0x8100]
    buf, offs, lens = PB.build(frames, PB.ETHER, ethertypes=types, fcs_len=4)
    pkts, l2 = pcap.index(buf)
    np.testing.assert_array_equal(l2, [OK, ARP, NOT_SUPPORT, OK, OK, SIZE, NOT_SUPPORT])
    np.testing.assert_array_equal(pkts["len"], [40, 0, 0, 0, 1500, 0, 0])
    assert pkts["offset"][0] == offs[0] and pkts["offset"][4] == offs[4]
    # a record shorter than an Ethernet header
    buf, _, _ = PB.build([b""], PB.ETHER, caplen_cut=[10])
    _, l2 = pcap.index(buf)
    np.testing.assert_array_equal(l2, [SIZE])


def test_truncated_records_are_the_captured_bytes(pcap):
    body = bytes(range(200))
    buf, offs, lens = PB.build([body, body], PB.ETHER, caplen_cut=[14 + 60, None])
    pkts, l2 = pcap.index(buf)
    np.testing.assert_array_equal(pkts["len"], [60, 200])
    np.testing.assert_array_equal(l2, [OK, OK])


def test_file_level_errors(pcap):
    import ctypes
    from tcp_amd import _lib
    L = _lib.pcap_lib()
    body = bytes(range(64))
    buf, offs, _ = PB.build([body] * 5, PB.ETHER)
    n = ctypes.c_uint32(0)
    # count only
    assert L.tcsum_pcap_index(buf, len(buf), None, None, 0, ctypes.byref(n)) == MEM and n.value == 5
    # too small an output: the first max_frames are indexed
    from tcp_amd import PKT_DTYPE
    pk = np.zeros(3, PKT_DTYPE)
    assert L.tcsum_pcap_index(buf, len(buf), pk.ctypes.data, None, 3, ctypes.byref(n)) == MEM
    assert n.value == 5 and (pk["offset"] == offs[:3]).all()
    # the file ends inside the last record / inside a record header
    for cut in (len(buf) - 10, len(buf) - (14 + 64) - 8):
        pk = np.zeros(5, pk.dtype)
        assert L.tcsum_pcap_index(buf[:cut], cut, pk.ctypes.data, None, 5, ctypes.byref(n)) == SIZE
        assert n.value == 4 and (pk["offset"][:4] == offs[:4]).all()
    # empty capture (header only)
    assert L.tcsum_pcap_index(buf[:24], 24, pk.ctypes.data, None, 5, ctypes.byref(n)) == OK and n.value == 0
    # not a savefile / too short / a pcapng SHB type on a classic body / unsupported link type
    assert L.tcsum_pcap_index(b"\0" * 64, 64, pk.ctypes.data, None, 5, ctypes.byref(n)) == PARAM
    assert L.tcsum_pcap_index(buf, 20, pk.ctypes.data, None, 5, ctypes.byref(n)) == PARAM
    assert L.tcsum_pcap_index(bytes.fromhex("0a0d0d0a") + buf[4:], len(buf), pk.ctypes.data, None, 5,
                              ctypes.byref(n)) == PARAM
    other = bytearray(buf)
    other[20:24] = (105).to_bytes(4, "little")  # IEEE 802.11
    assert L.tcsum_pcap_index(bytes(other), len(other), pk.ctypes.data, None, 5, ctypes.byref(n)) == NOT_SUPPORT
    assert L.tcsum_pcap_index(None, 0, None, None, 0, ctypes.byref(n)) == PARAM


@pytest.mark.parametrize("seed", range(4))
def test_parallel_walk_equals_sequential(pcap, monkeypatch, seed):
    """Large files are walked in pieces that find their own record boundary:
    with 1-4 KiB pieces (as many walkers as the host has, up to 16) the index
    equals the one-piece walk, also when payloads are full of fake record
    headers and when the file ends inside a record."""
    rng = np.random.default_rng(seed)
    n = 3000
    lens = rng.integers(0, 600, n)
    frames = []
    for i, L in enumerate(lens):
        f = bytearray(rng.integers(0, 256, L, dtype=np.uint8).tobytes())
        if seed % 2 and L >= 32:  # plant chains of plausible record headers in the payload
            for k in range(0, L - 16, 16):
                f[k: k + 16] = np.array([i, 7, (L - k) % 33, 40], "<u4").tobytes()
        frames.append(bytes(f))
    buf, offs, lens_exp = PB.build(frames, [PB.ETHER, PB.RAW, PB.NULL, PB.SLL][seed], big_endian=seed == 2)
    one = pcap.index(buf)
    np.testing.assert_array_equal(one[0]["offset"][one[1] == OK], offs[one[1] == OK])
    for kb in ("1", "2", "4"):
        monkeypatch.setenv("TCSUM_PCAP_PIECE_KB", kb)
        many = pcap.index(buf)
        np.testing.assert_array_equal(many[0], one[0])
        np.testing.assert_array_equal(many[1], one[1])
    # the file ends inside a record: the whole records before it, SIZE
    import ctypes
    from tcp_amd import _lib, PKT_DTYPE
    cut = int(offs[n // 2]) + 3
    for kb in (None, "1"):
        if kb:
            monkeypatch.setenv("TCSUM_PCAP_PIECE_KB", kb)
        else:
            monkeypatch.delenv("TCSUM_PCAP_PIECE_KB", raising=False)
        pk = np.zeros(n, PKT_DTYPE)
        got = ctypes.c_uint32(0)
        rc = _lib.pcap_lib().tcsum_pcap_index(buf[:cut], cut, pk.ctypes.data, None, n, ctypes.byref(got))
        assert rc == SIZE and got.value == n // 2
        np.testing.assert_array_equal(pk[: n // 2], one[0][: n // 2])


@pytest.mark.gpu
@pytest.mark.parametrize("link", [PB.RAW, PB.ETHER, PB.SLL])
def test_capture_rx_verify_golden(pcap, link):
    """The reference's rx verdicts, from a capture file verified in place:
    frames ether's is_pkt_ok rejects (> 1500 B of L3) get NET_ERR_SIZE
    before ipv4_in; every other frame the fixture's verdict, bit for bit."""
    cases, frames = golden_frames()
    buf, _, _ = PB.build(frames, link)
    verdict, l2, out, flags = pcap.rx_verify(np.frombuffer(buf, np.uint8))
    want = cases["verdict"].astype(np.int8)
    if link == PB.ETHER:
        want = np.where(cases["frame_len"] > 1500, SIZE, want).astype(np.int8)
    np.testing.assert_array_equal(verdict, want)
    reached = l2 == OK
    np.testing.assert_array_equal(flags[reached], cases["flags"][reached])


@pytest.mark.gpu
def test_capture_rx_verify_mixed_vs_oracle(pcap, oracle):
    """A 20,000-frame capture of configs[3]-style packets (tx-filled, then a
    few corrupted): verdicts equal the oracle's on the same L3 bytes."""
    from tcp_amd import workload
    b = workload.make_batch("mixed_rx", n=20000)
    dev, _ = workload.materialize(b)  # IPv4 packets generated in HBM, tx-filled like a sender
    arena = down(dev)
    rng = np.random.default_rng(11)
    frames = [arena[o: o + n].tobytes() for o, n in zip(b.descs["offset"], b.descs["len"])]
    for i in rng.choice(len(frames), 300, replace=False):
        f = bytearray(frames[i])
        f[rng.integers(0, len(f))] ^= 0x5A
        frames[i] = bytes(f)
    buf, offs, lens = PB.build(frames, PB.RAW, big_endian=True)
    verdict, l2, out, flags = pcap.rx_verify(np.frombuffer(buf, np.uint8))
    v3, _, _, _ = pcap.rx_verify(np.frombuffer(buf, np.uint8), devices=[0, 0, 0])  # sharded
    np.testing.assert_array_equal(v3, verdict)
    from tcp_amd import PKT_DTYPE
    pk = np.zeros(len(frames), PKT_DTYPE)
    pk["offset"], pk["len"] = offs, lens
    ev, ef = oracle.batch_ipv4_rx_verify(np.frombuffer(buf, np.uint8), pk, nthreads=8)
    np.testing.assert_array_equal(verdict, ev)
    assert (verdict == -13).sum() > 200  # the corruptions are seen


@pytest.mark.gpu
def test_c_pcap_verify(tmp_path):
    """tests/c/pcap_verify.c (INTEGRATION.md §4b in plain C) on a capture of
    the reference's rx fixtures: the per-frame verdicts it writes are the
    fixture's (Ethernet: frames over 1514 B get ether's NET_ERR_SIZE)."""
    import os
    import subprocess
    cases, frames = golden_frames()
    buf, _, _ = PB.build(frames, PB.ETHER)
    cap, res = tmp_path / "rx.pcap", tmp_path / "verdicts.bin"
    cap.write_bytes(buf)
    here = os.path.dirname(os.path.abspath(__file__))
    exe = os.path.join(here, "c", "build", "pcap_verify")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(here, "c")], check=True)
    r = subprocess.run([exe, str(cap), str(res)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    want = np.where(cases["frame_len"] > 1500, SIZE, cases["verdict"]).astype(np.int8)
    np.testing.assert_array_equal(np.fromfile(res, np.int8), want)
    assert r.stdout.startswith(f"{len(frames)} frames:")


@pytest.mark.gpu
@pytest.mark.parametrize("link", [PB.RAW, PB.ETHER])
def test_capture_tx_fill_golden(pcap, link):
    """A capture of the reference's tx fixture packets (tests/golden/ipv4_tx_*):
    filled in place, every frame that reaches ipv4_in holds exactly the bytes
    the reference's tx path produced; the others (Ethernet frames over 1514 B)
    and every record header are untouched."""
    cases, pin, pout = G.ipv4_tx_cases()
    before = [pin[o: o + n].tobytes() for o, n in zip(cases["pool_off"], cases["frame_len"])]
    after = [pout[o: o + n].tobytes() for o, n in zip(cases["pool_off"], cases["frame_len"])]
    buf, offs, lens = PB.build(before, link)
    a = np.frombuffer(bytearray(buf), np.uint8)
    l2, flags = pcap.tx_fill(a)
    filled = l2 == OK
    if link == PB.RAW:
        assert filled.all()
    else:
        np.testing.assert_array_equal(filled, cases["frame_len"] <= 1500)
    np.testing.assert_array_equal(flags[filled], cases["flags"][filled])
    want, _, _ = PB.build([after[i] if filled[i] else before[i] for i in range(len(before))], link)
    assert a.tobytes() == want


@pytest.mark.parametrize("big_endian", [False, True])
@pytest.mark.parametrize("block", ["epb", "spb", "pb"])
def test_pcapng_index(pcap, big_endian, block):
    """pcapng: Enhanced / Simple / obsolete Packet Blocks, either byte order,
    other block types skipped; descriptors point at each frame's IPv4 bytes."""
    cases, frames = golden_frames()
    frames = [f for f in frames if len(f) <= 1500]
    buf, offs, lens = PB.build_ng(frames, (PB.ETHER,), big_endian=big_endian, block=block)
    pkts, l2 = pcap.index(buf)
    np.testing.assert_array_equal(l2, OK)
    np.testing.assert_array_equal(pkts["offset"], offs)
    np.testing.assert_array_equal(pkts["len"], lens)


def test_pcapng_interfaces_sections_fcs(pcap):
    """Per-interface link types (Ethernet, raw, cooked, an unsupported one),
    several sections (each resets the interface table), an FCS length option
    in bits (if_fcslen)."""
    body = bytes(range(60))
    n = 40
    iface = [i % 4 for i in range(n)]
    links = (PB.ETHER, PB.RAW, PB.SLL, 105)  # 105: IEEE 802.11, not read here
    buf, offs, lens = PB.build_ng([body] * n, links, iface_of=iface, sections=3, fcs_bits=32)
    pkts, l2 = pcap.index(buf)
    want = np.array([NOT_SUPPORT if i == 3 else OK for i in iface], np.int8)
    np.testing.assert_array_equal(l2, want)
    ok = want == OK
    np.testing.assert_array_equal(pkts["offset"][ok], offs[ok])
    np.testing.assert_array_equal(pkts["len"][ok], 60)


def test_pcapng_errors(pcap):
    import ctypes
    from tcp_amd import _lib, PKT_DTYPE
    L = _lib.pcap_lib()
    body = bytes(range(64))
    buf, offs, _ = PB.build_ng([body] * 5, (PB.ETHER,), extra_blocks=False)
    pk = np.zeros(5, PKT_DTYPE)
    n = ctypes.c_uint32(0)
    assert L.tcsum_pcap_index(buf, len(buf), None, None, 0, ctypes.byref(n)) == MEM and n.value == 5
    assert L.tcsum_pcap_index(buf[:-6], len(buf) - 6, pk.ctypes.data, None, 5, ctypes.byref(n)) == SIZE
    assert n.value == 4 and (pk["offset"][:4] == offs[:4]).all()
    bad = bytearray(buf)
    bad[-1] ^= 0x40  # trailing block length differs from the leading one
    assert L.tcsum_pcap_index(bytes(bad), len(bad), pk.ctypes.data, None, 5, ctypes.byref(n)) == PARAM
    bad = bytearray(buf)
    bad[8:12] = b"\0\0\0\0"  # byte-order magic
    assert L.tcsum_pcap_index(bytes(bad), len(bad), pk.ctypes.data, None, 5, ctypes.byref(n)) == PARAM


@pytest.mark.gpu
def test_pcapng_rx_verify_golden(pcap):
    """The reference's rx verdicts from a pcapng capture (raw-IPv4 interface)."""
    cases, frames = golden_frames()
    buf, _, _ = PB.build_ng(frames, (PB.RAW,))
    verdict, l2, out, flags = pcap.rx_verify(np.frombuffer(buf, np.uint8))
    np.testing.assert_array_equal(verdict, cases["verdict"].astype(np.int8))


@pytest.mark.parametrize("seed", range(4))
def test_pcapng_parallel_walk(pcap, monkeypatch, seed):
    """Large pcapng files are walked in parallel pieces from the first packet
    block on: with 1-4 KiB pieces the index equals the one-piece walk, with
    fake blocks planted in payloads, with statistics blocks between packets,
    and -- falling back to the sequential walk -- with several sections."""
    import struct
    rng = np.random.default_rng(100 + seed)
    n = 2500
    frames = []
    for i in range(n):
        L = int(rng.integers(0, 500))
        f = bytearray(rng.integers(0, 256, L, dtype=np.uint8).tobytes())
        if seed % 2 and L > 48:  # a fake EPB (consistent lengths) inside the payload
            fake = struct.pack("<IIIIIII", 6, 48, 0, 0, 0, 16, 16) + bytes(16) + struct.pack("<I", 48)
            k = int(rng.integers(0, L - 48))
            f[k: k + 48] = fake
        frames.append(bytes(f))
    links = (PB.ETHER, PB.RAW)
    iface = [int(x) for x in rng.integers(0, 2, n)]
    for sections in (1, 3):
        buf, offs, lens = PB.build_ng(frames, links, iface_of=iface, big_endian=seed == 2,
                                      block=["epb", "pb", "epb", "epb"][seed], sections=sections)
        monkeypatch.delenv("TCSUM_PCAP_PIECE_KB", raising=False)
        one = pcap.index(buf)
        np.testing.assert_array_equal(one[0]["offset"], offs)
        np.testing.assert_array_equal(one[0]["len"], lens)
        for kb in ("1", "4"):
            monkeypatch.setenv("TCSUM_PCAP_PIECE_KB", kb)
            many = pcap.index(buf)
            np.testing.assert_array_equal(many[0], one[0])
            np.testing.assert_array_equal(many[1], one[1])


@pytest.mark.gpu
def test_cli_verify_and_fill(tmp_path):
    """python -m tcp_amd.pcap: counts per verdict; --fill writes the capture
    with the reference's tx bytes."""
    import os
    import subprocess
    import sys
    cases, pin, pout = G.ipv4_tx_cases()
    before = [pin[o: o + n].tobytes() for o, n in zip(cases["pool_off"], cases["frame_len"])]
    after = [pout[o: o + n].tobytes() for o, n in zip(cases["pool_off"], cases["frame_len"])]
    buf, _, _ = PB.build(before, PB.RAW)
    src, dst = tmp_path / "in.pcap", tmp_path / "out.pcap"
    src.write_bytes(buf)
    r = subprocess.run([sys.executable, "-m", "tcp_amd.pcap", str(src), "--fill", str(dst)],
                       capture_output=True, text=True, timeout=120,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith(f"{len(before)} frames: ")
    want, _, _ = PB.build(after, PB.RAW)
    assert dst.read_bytes() == want


def test_pcapng_parallel_walk_same_acceptance(pcap, monkeypatch):
    """The parallel pcapng walk accepts exactly what the one-piece walk
    accepts: a header-region block whose trailing length disagrees is refused
    by both; a Simple Packet Block too short for its length word is an empty
    frame for both."""
    import struct
    rng = np.random.default_rng(7)
    frames = [rng.integers(0, 256, int(rng.integers(20, 300)), dtype=np.uint8).tobytes() for _ in range(3000)]
    buf, offs, lens = PB.build_ng(frames, (PB.RAW,), block="spb", extra_blocks=False)
    # (a) corrupt the IDB's trailing length (the IDB follows the 28-byte SHB)
    idb_len = struct.unpack_from("<I", buf, 28 + 4)[0]
    bad = bytearray(buf)
    struct.pack_into("<I", bad, 28 + idb_len - 4, idb_len + 4)
    results = []
    for kb in (None, "1"):
        if kb is None:
            monkeypatch.delenv("TCSUM_PCAP_PIECE_KB", raising=False)
        else:
            monkeypatch.setenv("TCSUM_PCAP_PIECE_KB", kb)
        with pytest.raises(Exception):
            pcap.index(bytes(bad))
    # (b) a 12-byte SPB (no length word) in the middle of the packet blocks
    k = int(offs[1500]) - 12  # the SPB of frame 1500 starts 12 bytes before its data
    short = struct.pack("<III", 3, 12, 12)
    good = bytes(buf[:k]) + short + bytes(buf[k:])
    for kb in (None, "1", "4"):
        if kb is None:
            monkeypatch.delenv("TCSUM_PCAP_PIECE_KB", raising=False)
        else:
            monkeypatch.setenv("TCSUM_PCAP_PIECE_KB", kb)
        results.append(pcap.index(good))
    for r in results[1:]:
        np.testing.assert_array_equal(r[0], results[0][0])
        np.testing.assert_array_equal(r[1], results[0][1])
    assert results[0][0].size == 3001 and results[0][0]["len"][1500] == 0
