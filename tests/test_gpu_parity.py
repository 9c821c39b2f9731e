"""Parity of the HIP path with the reference, on an MI355X.

Every call goes through libtcsum.so's C ABI.  Expected values come from
  * tests/golden/ -- outputs of the reference's own checksum16 /
    pktbuf_checksum16 / checksum_peso (net/src/tools.c:24-75,
    net/src/pktbuf.c:646-670) on recorded inputs, and
  * the CPU oracle (oracle/, pinned to those fixtures) on seeded inputs.
The bar is bit-exact: these are 16-bit integer results.
"""
from devcopy import down, up
import ctypes
import os

import numpy as np
import pytest

import golden_io as G

pytestmark = pytest.mark.gpu

# every shape the router can pick (libtcsum.so instantiates these and no others)
GEOMS_SEG = [(4, 1), (4, 2), (8, 4), (16, 3), (16, 4), (16, 6), (16, 8), (32, 6),
             (256, 16),  # one range per workgroup: k_segments_wg
             (1024, 4)]  # one range per 16-wave workgroup: k_segments_wgx<16, 32, 4> (TSO)
GEOMS_IP = [(16, 1), (16, 2), (16, 3), (16, 4), (16, 6), (16, 8), (32, 6), (64, 4), (64, 16)]


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


@pytest.fixture
def knobs(tc):
    """Set route knobs (include/tcsum_debug.h) for one test; every knob set
    goes back to the router's choice afterwards."""
    touched = set()

    def set_knobs(**kw):
        for k, v in kw.items():
            tc.debug_set(k, v)
            touched.add(k)
    yield set_knobs
    for k in touched:
        tc.debug_set(k, -1)


@pytest.fixture
def geometry(knobs):
    def set_geometry(g, u):
        knobs(lanes=g, loads=u)
    return set_geometry


def to_dev(torch, a: np.ndarray, pad: int = 64):
    t = torch.zeros(a.nbytes + pad, dtype=torch.uint8)
    t[: a.nbytes] = torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1))
    return up(t)


def test_native_library_is_loaded(tc):
    assert tc.checksum16(0, b"\xff\xff", 2, 0, 1) == 0
    maps = open("/proc/self/maps").read()
    assert "libtcsum.so" in maps


# ------------------------------------------------------------ drop-in trio

def test_kats(tc):
    k = G.kat_inputs()
    h, e = k["KAT-1"]
    assert tc.checksum16(0, h, 20, 0, 1) == e == 0x61B8
    filled = bytearray(h)
    filled[10:12] = e.to_bytes(2, "little")
    assert tc.checksum16(0, bytes(filled), 20, 0, 1) == 0
    b, e = k["KAT-2"]
    assert tc.checksum16(0, b, 999, 0, 1) == e
    buf = tc.PktBuf([b[i: i + 127] for i in range(0, 999, 127)])
    assert tc.pktbuf_checksum16(buf, 999, 0, 1) == e == 0x8EE9
    b, e = k["KAT-3"]
    buf = tc.PktBuf([b[i: i + 127] for i in range(0, 999, 127)])
    got = tc.checksum_peso(buf, tc.IpAddr.v4([192, 168, 74, 3]), tc.IpAddr.v4([192, 168, 74, 2]), 6)
    assert got == e == 0x4AD0
    assert tc.checksum16(0, bytes(4), 4, 0, 1) == 0xFFFF
    assert tc.checksum16(0, b"\xff\xff", 2, 0, 1) == 0


def test_checksum16_golden(tc):
    pool = G.pool()
    bad = []
    for c in G.flat_cases():
        off, n = int(c["pool_off"]), int(c["len"])
        got = tc.checksum16(int(c["offset"]), pool[off: off + n], n, int(c["pre_sum"]), int(c["complement"]))
        if got != int(c["expected"]):
            bad.append((dict(zip(c.dtype.names, c.tolist())), got))
    assert not bad, bad[:5]


def test_pktbuf_checksum16_golden(tc):
    """Result AND cursor side effect (pktbuf.c:665) match the reference."""
    pool = G.pool()
    cases, blocks = G.pktbuf_cases()
    for c in cases:
        buf = tc.PktBuf([p.tobytes() for p in G.case_blocks(c, blocks, pool)])
        if int(c["seek"]):
            buf.seek(int(c["seek"]))
        got = tc.pktbuf_checksum16(buf, int(c["len"]), int(c["pre_sum"]), int(c["complement"]))
        assert got == int(c["expected"]), c
        pos, blk, boff = buf.cursor()
        exp_blk = None if int(c["final_blk"]) == G.NO_BLOCK else int(c["final_blk"])
        assert (pos, blk) == (int(c["final_pos"]), exp_blk), c
        if blk is not None:
            assert boff == int(c["final_blk_off"]), c


def test_checksum_peso_golden(tc):
    pool = G.pool()
    cases, blocks = G.peso_cases()
    for c in cases:
        buf = tc.PktBuf([p.tobytes() for p in G.case_blocks(c, blocks, pool)])
        buf.seek(min(3, int(c["total"]) - 1))  # checksum_peso resets the cursor itself
        got = tc.checksum_peso(buf, tc.IpAddr.v4(c["dst"].tobytes()), tc.IpAddr.v4(c["src"].tobytes()),
                               int(c["proto"]))
        assert got == int(c["expected"]), c
        pos, blk, _ = buf.cursor()
        assert pos == int(c["final_pos"]) == int(c["total"]) and blk is None


def test_dropin_golden_with_descriptor_in_pinned_memory(tc):
    """Debug knob args_launch = 0: every drop-in call takes the path with its
    descriptor in pinned memory (the one calls above 16 KiB always take);
    the same reference results and cursors as the kernel-argument path."""
    tc.debug_set("args_launch", 0)
    try:
        test_kats(tc)
        test_checksum16_golden(tc)
        test_pktbuf_checksum16_golden(tc)
        test_checksum_peso_golden(tc)
    finally:
        tc.debug_set("args_launch", -1)


@pytest.mark.parametrize("args_launch", ["1", "0"])
def test_pktbuf_checksum16_16k_to_64k(tc, oracle, knobs, args_launch):
    """pktbuf_checksum16 on chains of 16-64 KiB (the reference's pool stops
    at 12,700 B, so its goldens do; parity here is against the oracle, which
    those goldens pin): irregular 1..127-byte blocks, a seek, any length up to
    what is left (and one past it: 0, pktbuf.c:650-655), any pre_sum and
    complement; result and final cursor (pos, block)."""
    knobs(args_launch=int(args_launch))
    rng = np.random.default_rng(1616 + int(args_launch))
    for case in range(60):
        total = int(rng.integers(16 << 10, (64 << 10) + 1))
        sizes = []
        while sum(sizes) < total:
            sizes.append(int(min(rng.integers(1, 128), total - sum(sizes))))
        data = rng.integers(0, 256, total, dtype=np.uint8)
        if case % 7 == 0:
            data[:] = 0xFF
        pieces, at = [], 0
        for s in sizes:
            pieces.append(data[at: at + s].tobytes())
            at += s
        buf = tc.PktBuf(pieces)
        seek = int(rng.integers(0, min(total, 3000)))
        if seek:
            buf.seek(seek)
        left = total - seek
        length = left + 1 if case % 11 == 5 else int(rng.integers(0, left + 1))
        pre, comp = int(rng.integers(0, 1 << 31)), int(rng.integers(0, 2))
        # the oracle's pieces from the cursor: the rest of the cursor's block, then whole blocks
        pos, blk, boff = buf.cursor()
        rest = [pieces[blk][boff:]] + pieces[blk + 1:] if blk is not None else []
        want = oracle.pieces_checksum16(rest, length, pre, comp)
        got = tc.pktbuf_checksum16(buf, length, pre, comp)
        assert got == want, (case, total, seek, length)
        end = seek + (length if length <= left else 0)
        assert buf.cursor()[0] == end, (case, buf.cursor(), end)


def test_reference_stack_objects_link_against_libtcsum(tc):
    """oracle/_ref/dropin_stack: the reference's own pktbuf.o/tools.o (checksum
    definitions localized, as INTEGRATION.md patches them out) linked with
    libtcsum.so, replaying every pktbuf/peso golden case through the reference's
    own chain and cursor code."""
    import subprocess
    exe = os.path.join(os.path.dirname(G.GOLDEN), "..", "oracle", "_ref", "dropin_stack")
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref not built (needs /root/reference at build time)")
    r = subprocess.run([exe, G.GOLDEN], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "2749/2749" in r.stdout


def test_c_host_batch_demo(tc):
    """tests/c/batch_demo.c: a plain C host (HIP C API + libtcsum.so) runs the
    batch and end-to-end paths, and a tx fill captured in a hipGraph through
    the C API (tcsum_batch_ipv4_tx_fill_scratch); the CPU oracle checks every
    result."""
    import subprocess
    exe = os.path.join(os.path.dirname(G.GOLDEN), "c", "build", "batch_demo")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.dirname(os.path.dirname(exe))], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 mismatches" in r.stdout


# ------------------------------------------------------------ batches

def peso_descs(tc, cases):
    d = np.zeros(cases.size, tc.PESO_DTYPE)
    d["offset"] = cases["pool_off"]
    d["len"] = cases["total"]
    d["src"] = cases["src"]
    d["dst"] = cases["dst"]
    d["protocol"] = cases["proto"]
    return d


@pytest.mark.parametrize("g,u", GEOMS_SEG)
def test_batch_peso_golden(tc, torch, geometry, g, u):
    geometry(g, u)
    pool = G.pool()
    cases, _ = G.peso_cases()
    arena = to_dev(torch, pool)
    d = peso_descs(tc, cases)
    out = tc.batch_peso(arena, tc.descs_to_device(d), d.size, int(d["len"].sum()))
    np.testing.assert_array_equal(down(out), cases["expected"].astype(np.uint16))



@pytest.mark.parametrize("xg", [1, 2, 3, 5, 64])
def test_xcd_block_order_golden(tc, torch, geometry, knobs, xg):
    """The XCD-grouped workgroup order (debug knob xcd) is a bijection on the grid:
    with groups small enough that the golden batches hold whole 8*xg groups
    AND a tail group, every segment / packet still gets exactly its own result."""
    knobs(xcd=xg)
    geometry(4, 2)
    pool = G.pool()
    cases, _ = G.peso_cases()
    d = peso_descs(tc, cases)
    out = torch.empty(d.size, dtype=torch.uint16, device="cuda")
    out.view(torch.int16).fill_(-0x5556)  # 0xAAAA: a result nobody wrote shows up
    tc.batch_peso(to_dev(torch, pool), tc.descs_to_device(d), d.size, out=out)
    np.testing.assert_array_equal(down(out), cases["expected"].astype(np.uint16))
    geometry(16, 4)
    cases, ipool = G.ipv4_rx_cases()
    pk = G.pkt_descs(cases, tc.PKT_DTYPE)
    verdict, flags = tc.batch_ipv4_rx_verify(to_dev(torch, ipool), tc.descs_to_device(pk), cases.size)
    np.testing.assert_array_equal(down(verdict), cases["verdict"])
    np.testing.assert_array_equal(down(flags), cases["flags"])
    cases, pin, pout = G.ipv4_tx_cases()
    arena = to_dev(torch, pin)
    tc.batch_ipv4_tx_fill(arena, tc.descs_to_device(G.pkt_descs(cases, tc.PKT_DTYPE)), cases.size)
    np.testing.assert_array_equal(down(arena)[: pout.size], pout)

@pytest.mark.parametrize("g,u", [(32, 6), (16, 4), (1024, 4)])
def test_batch_segments_golden(tc, torch, geometry, g, u):
    """pktbuf_checksum16 cases (from the cursor) and even-offset checksum16 cases
    with 16-bit pre_sum, where the two routines agree, as one batch each."""
    geometry(g, u)
    pool = G.pool()
    cases, _ = G.pktbuf_cases()
    keep = cases[(cases["len"] > 0) & (cases["len"] <= cases["total"] - cases["seek"])]
    flat = G.flat_cases()
    fkeep = flat[(flat["offset"] % 2 == 0) & (flat["pre_sum"] <= 0xFFFF)]
    arena = to_dev(torch, pool)
    for comp in (0, 1):
        k = keep[keep["complement"] == comp]
        f = fkeep[fkeep["complement"] == comp]
        s = np.zeros(k.size + f.size, tc.SEG_DTYPE)
        s["offset"][: k.size] = k["pool_off"].astype(np.uint64) + k["seek"]
        s["len"][: k.size] = k["len"]
        s["pre_sum"][: k.size] = k["pre_sum"].view(np.uint32)
        s["offset"][k.size:] = f["pool_off"]
        s["len"][k.size:] = f["len"]
        s["pre_sum"][k.size:] = f["pre_sum"]
        exp = np.concatenate([k["expected"], f["expected"]]).astype(np.uint16)
        out = tc.batch_segments(arena, tc.descs_to_device(s), s.size, comp, int(s["len"].sum()))
        np.testing.assert_array_equal(down(out), exp)


@pytest.mark.parametrize("g,u", GEOMS_IP)
def test_batch_ipv4_golden(tc, torch, geometry, g, u):
    geometry(g, u)
    cases, ipool = G.ipv4_cases()
    arena = to_dev(torch, ipool)
    pk = np.zeros(cases.size, tc.PKT_DTYPE)
    pk["offset"] = cases["pool_off"]
    pk["len"] = cases["frame_len"]
    out, flags = tc.batch_ipv4(arena, tc.descs_to_device(pk), pk.size, int(pk["len"].sum()))
    out = down(out)
    np.testing.assert_array_equal(out & 0xFFFF, cases["ip"])
    np.testing.assert_array_equal(out >> 16, cases["l4"])
    np.testing.assert_array_equal(down(flags), cases["flags"])


@pytest.mark.parametrize("mean", [0, 64, 300, 1500, 9000, 70000])
def test_batch_ipv4_every_picked_geometry(tc, torch, mean):
    """The length hint only changes the lane mapping, never the result."""
    cases, ipool = G.ipv4_cases()
    arena = to_dev(torch, ipool)
    pk = np.zeros(cases.size, tc.PKT_DTYPE)
    pk["offset"] = cases["pool_off"]
    pk["len"] = cases["frame_len"]
    out, flags = tc.batch_ipv4(arena, tc.descs_to_device(pk), pk.size, mean * pk.size)
    out = down(out)
    np.testing.assert_array_equal(out & 0xFFFF, cases["ip"])
    np.testing.assert_array_equal(out >> 16, cases["l4"])
    np.testing.assert_array_equal(down(flags), cases["flags"])


@pytest.mark.parametrize("mean", [0, 20, 64, 300, 1500, 9000, 70000])
def test_batch_peso_every_picked_geometry(tc, torch, mean):
    pool = G.pool()
    cases, _ = G.peso_cases()
    arena = to_dev(torch, pool)
    d = peso_descs(tc, cases)
    out = tc.batch_peso(arena, tc.descs_to_device(d), d.size, mean * d.size)
    np.testing.assert_array_equal(down(out), cases["expected"].astype(np.uint16))


def test_ipv4_odd_arena_base(tc, torch):
    """Same packets one byte further into the arena: address parity flips."""
    cases, ipool = G.ipv4_cases()
    arena = to_dev(torch, np.concatenate([np.zeros(1, np.uint8), ipool]))
    pk = np.zeros(cases.size, tc.PKT_DTYPE)
    pk["offset"] = cases["pool_off"].astype(np.uint64) + 1
    pk["len"] = cases["frame_len"]
    out, flags = tc.batch_ipv4(arena, tc.descs_to_device(pk), pk.size)
    out = down(out)
    np.testing.assert_array_equal(out & 0xFFFF, cases["ip"])
    np.testing.assert_array_equal(out >> 16, cases["l4"])
    np.testing.assert_array_equal(down(flags), cases["flags"])


TX_FORMS = ["fused", "deferred", "deferred_cold"]


def set_tx_form(knobs, form):
    """The forms of the in-place tx fill: stores in the kernel
    (k_ipv4<IP_TX>) or deferred to k_tx_scatter, which by default first
    loads the dword under each field (debug "tx_warm"; "deferred_cold"
    stores without it)."""
    knobs(tx_split=0 if form == "fused" else 1, tx_warm=0 if form == "deferred_cold" else -1)


@pytest.mark.parametrize("form", TX_FORMS)
@pytest.mark.parametrize("g,u", [(16, 1), (16, 4), (16, 8), (32, 6), (64, 4), (64, 16)])
def test_batch_ipv4_tx_fill_golden(tc, torch, geometry, knobs, g, u, form):
    """In-place fill == the reference's tx path on the same packets, byte for
    byte, in every form of the fill."""
    geometry(g, u)
    set_tx_form(knobs, form)
    cases, pin, pout = G.ipv4_tx_cases()
    arena = to_dev(torch, pin)
    d = tc.descs_to_device(G.pkt_descs(cases, tc.PKT_DTYPE))
    flags = tc.batch_ipv4_tx_fill(arena, d, cases.size, int(cases["frame_len"].sum()))
    np.testing.assert_array_equal(down(arena)[: pout.size], pout)
    np.testing.assert_array_equal(down(flags), cases["flags"])
    flags = tc.batch_ipv4_tx_fill(arena, d, cases.size)  # idempotent: fields read as zero
    np.testing.assert_array_equal(down(arena)[: pout.size], pout)


@pytest.mark.parametrize("form", TX_FORMS)
@pytest.mark.parametrize("g,u", [(16, 1), (16, 6), (32, 6), (64, 4), (64, 16)])
def test_batch_ipv4_tx_fill_stack_golden(tc, torch, geometry, knobs, g, u, form):
    """Frames the reference stack itself transmitted (udp_out, send_out,
    icmpv4_out, ipv4_out, ip_frag_out; oracle/stack_gen.c) with their filled
    fields junked: the in-place fill (every form) gives the reference's frames
    back, byte for byte, and the offload form + host apply gives the same
    bytes."""
    geometry(g, u)
    set_tx_form(knobs, form)
    cases, pin, pout = G.stack_tx_cases()
    pk = G.pkt_descs(cases, tc.PKT_DTYPE)
    arena = to_dev(torch, pin)
    d = tc.descs_to_device(pk)
    flags = tc.batch_ipv4_tx_fill(arena, d, cases.size, int(cases["frame_len"].sum()))
    np.testing.assert_array_equal(down(arena)[: pout.size], pout)
    np.testing.assert_array_equal(down(flags), cases["flags"])
    arena = to_dev(torch, pin)
    out, flags = tc.batch_ipv4_tx_offload(arena, d, cases.size, int(cases["frame_len"].sum()))
    host = pin.copy()
    tc.tx_apply_batch(host, pk, down(out), down(flags))
    np.testing.assert_array_equal(host[: pout.size], pout)


@pytest.mark.parametrize("g,u", [(16, 1), (32, 6), (64, 4), (64, 16)])
def test_batch_ipv4_tx_offload_golden(tc, torch, geometry, g, u):
    """tx offload: the packets stay untouched on the device, and the host
    applying out/flags gives the reference's filled frames byte for byte;
    out is the word tx fill reports for the same packets."""
    geometry(g, u)
    cases, pin, pout = G.ipv4_tx_cases()
    arena = to_dev(torch, pin)
    d = tc.descs_to_device(G.pkt_descs(cases, tc.PKT_DTYPE))
    out, flags = tc.batch_ipv4_tx_offload(arena, d, cases.size, int(cases["frame_len"].sum()))
    np.testing.assert_array_equal(down(arena)[: pin.size], pin)
    np.testing.assert_array_equal(down(flags), cases["flags"])
    host = pin.copy()
    tc.tx_apply_batch(host, G.pkt_descs(cases, tc.PKT_DTYPE), down(out), down(flags))
    np.testing.assert_array_equal(host[: pout.size], pout)
    fill_out = torch.empty(cases.size, dtype=torch.uint32, device="cuda")
    tc.batch_ipv4_tx_fill(arena, d, cases.size, out=fill_out)
    np.testing.assert_array_equal(down(out), down(fill_out))


@pytest.mark.parametrize("form", TX_FORMS)
@pytest.mark.parametrize("top", [160, 700])
@pytest.mark.parametrize("layout", ["packed", "gaps", "shuffled"])
def test_tx_fill_neighbours(tc, torch, oracle, knobs, layout, top, form):
    """Both fill forms on small packets (28-160 B: neighbours' fields share
    64-B sectors and 128-B lines; 28-700 B: a mix), back to back at an odd
    base, with gaps between some (bytes of no packet: must stay untouched), or
    with the descriptors shuffled: every byte of the arena equals the
    oracle's fill."""
    set_tx_form(knobs, form)
    rng = np.random.default_rng({"packed": 1, "gaps": 2, "shuffled": 3}[layout] + top)
    n = 20000
    proto = rng.choice([6, 17, 1], n)
    lo = np.where(proto == 6, 40, np.where(proto == 17, 28, 24))
    lens = rng.integers(lo, top + 1)
    gap = rng.integers(0, 40, n) * (rng.random(n) < 0.3) if layout == "gaps" else np.zeros(n, np.int64)
    offs = 7 + np.concatenate([[0], np.cumsum(lens + gap)[:-1]])
    arena = rng.integers(0, 256, int(offs[-1] + lens[-1] + 200), dtype=np.uint8)
    for i in range(n):
        o, L = int(offs[i]), int(lens[i])
        arena[o] = 0x45
        arena[o + 2: o + 4] = (L >> 8, L & 0xFF)
        arena[o + 6] &= 0x40  # DF at most: not a fragment
        arena[o + 7] = 0
        arena[o + 9] = proto[i]
    pk = np.zeros(n, tc.PKT_DTYPE)
    pk["offset"], pk["len"] = offs, lens
    if layout == "shuffled":
        pk = pk[rng.permutation(n)]
    want = arena.copy()
    wfl = oracle.batch_ipv4_tx_fill(want, pk)
    d_arena = to_dev(torch, arena)
    fl = tc.batch_ipv4_tx_fill(d_arena, tc.descs_to_device(pk), n, int(lens.sum()))
    np.testing.assert_array_equal(down(fl), wfl)
    np.testing.assert_array_equal(down(d_arena)[: arena.size], want)


def test_tx_offload_full_mixed(tc, torch, knobs):
    """configs[3] at full size: offload + host apply == in-place fill, every
    byte, in the default form at this size and in the other two; the fill's
    `out` equals the offload's."""
    from tcp_amd import workload
    b = workload.make_batch("mixed")
    arena, descs = workload.materialize(b)
    unfilled = arena.clone()
    out, flags = tc.batch_ipv4_tx_offload(arena, descs, b.n, b.total_bytes)
    host = torch.from_numpy(down(arena))
    tc.tx_apply_batch(host.numpy(), b.descs, down(out), down(flags))
    want = host.to(arena.device)
    del host
    fill_out = torch.empty_like(out)
    tc.batch_ipv4_tx_fill(arena, descs, b.n, b.total_bytes, out=fill_out, want_flags=False)
    torch.cuda.synchronize()
    assert torch.equal(arena, want) and torch.equal(fill_out, out)
    for form in TX_FORMS:
        arena.copy_(unfilled)
        set_tx_form(knobs, form)
        tc.batch_ipv4_tx_fill(arena, descs, b.n, b.total_bytes, want_flags=False)
        torch.cuda.synchronize()
        assert torch.equal(arena, want), form


@pytest.mark.parametrize("g,u", [(16, 1), (16, 4), (16, 8), (32, 6), (64, 4), (64, 16)])
def test_batch_ipv4_rx_verify_golden(tc, torch, oracle, geometry, g, u):
    geometry(g, u)
    cases, pool = G.ipv4_rx_cases()
    arena = to_dev(torch, pool)
    pk = G.pkt_descs(cases, tc.PKT_DTYPE)
    out = torch.empty(cases.size, dtype=torch.uint32, device="cuda")
    verdict, flags = tc.batch_ipv4_rx_verify(arena, tc.descs_to_device(pk), cases.size, out=out)
    np.testing.assert_array_equal(down(verdict), cases["verdict"])
    np.testing.assert_array_equal(down(flags), cases["flags"])
    exp, _ = oracle.batch_ipv4(pool, pk)
    np.testing.assert_array_equal(down(out), exp)


def test_tx_then_rx_full_mixed(tc, torch, oracle):
    """configs[3] at full size: fill on the GPU, verify on the GPU (all OK),
    corrupt 2,000 packets, verify again; the oracle agrees on every packet."""
    from tcp_amd import workload
    b = workload.make_batch("mixed")
    arena, descs = workload.materialize(b)
    tc.batch_ipv4_tx_fill(arena, descs, b.n, b.total_bytes)
    verdict, _ = tc.batch_ipv4_rx_verify(arena, descs, b.n, b.total_bytes)
    assert (down(verdict) == 0).all()
    rng = np.random.default_rng(5)
    bad = rng.choice(b.n, 2000, replace=False)
    pos = (b.descs["offset"][bad] + 20 + (rng.integers(0, 1 << 30, bad.size) % (b.descs["len"][bad] - 20))).astype(np.int64)
    idx = up(torch.from_numpy(pos))
    arena[idx] ^= 0x04
    verdict, flags = tc.batch_ipv4_rx_verify(arena, descs, b.n, b.total_bytes)
    v = down(verdict)
    assert (v[bad] == -13).mean() > 0.99 and (np.delete(v, bad) == 0).all()
    host = down(arena)
    ev, ef = oracle.batch_ipv4_rx_verify(host, b.descs, nthreads=16)
    np.testing.assert_array_equal(v, ev)
    np.testing.assert_array_equal(down(flags), ef)


# ------------------------------------------------- seeded batches vs oracle

def run_config(tc, torch, config, n):
    from tcp_amd import workload
    b = workload.make_batch(config, rank=1, n=n)
    arena, descs = workload.materialize(b)
    if b.kind == "peso":
        out = tc.batch_peso(arena, descs, b.n, b.total_bytes)
    else:
        out, flags = tc.batch_ipv4(arena, descs, b.n, b.total_bytes)
    torch.cuda.synchronize()
    return b, arena, out


@pytest.mark.parametrize("config,n", [("mtu", 50000), ("tso", 600), ("mixed", 20000), ("mixed_aligned", 20000)])
def test_config_vs_oracle(tc, torch, oracle, config, n):
    b, arena, out = run_config(tc, torch, config, n)
    host = down(arena)
    # the device generator is the oracle's stream
    np.testing.assert_array_equal(host[:4096], oracle.synth_fill(b.byte_base, 4096, b.seed)[:4096]
                                  if b.kind == "peso" else host[:4096])
    if b.kind == "peso":
        exp = oracle.batch_peso(host, b.descs, nthreads=8)
        np.testing.assert_array_equal(down(out), exp)
    else:
        exp, fl = oracle.batch_ipv4(host, b.descs, nthreads=8)
        np.testing.assert_array_equal(down(out), exp)
        assert (fl == 0).all()  # synthetic headers are well formed


@pytest.mark.parametrize("g,u", GEOMS_SEG)
def test_geometries_vs_oracle(tc, torch, oracle, geometry, g, u):
    geometry(g, u)
    b, arena, out = run_config(tc, torch, "mtu", 4096)
    exp = oracle.batch_peso(down(arena), b.descs, nthreads=8)
    np.testing.assert_array_equal(down(out), exp)


def test_edge_segments(tc, torch, oracle):
    """Empty, 1-byte, odd starts, all-zero, all-0xFF, sums folding to 0xFFFF,
    a segment ending on the allocation's last byte, and a 32 MiB segment."""
    rng = np.random.default_rng(7)
    size = (32 << 20) + 8192
    host = rng.integers(0, 256, size, dtype=np.uint8)
    host[1000:3000] = 0
    host[4000:6000] = 0xFF
    # 0xFF00 + 0x00FF = 0xFFFF: folds to 0xFFFF, complement 0
    host[7000:7004] = [0x00, 0xFF, 0xFF, 0x00]
    segs = [(0, 0), (5, 0), (9, 1), (10, 1), (11, 2), (12, 3), (1000, 2000), (1001, 1998), (4000, 2000),
            (4001, 1999), (7000, 4), (7001, 3), (13, 65535), (17, 65536), (19, 65537), (8191, 1),
            (size - 1, 1), (size - 17, 17), (size - 100, 100), (8192, 32 << 20)]
    segs += [(int(o), int(n)) for o, n in zip(rng.integers(0, size - 70000, 300), rng.integers(0, 70000, 300))]
    s = np.zeros(len(segs), tc.SEG_DTYPE)
    s["offset"] = [o for o, _ in segs]
    s["len"] = [n for _, n in segs]
    s["pre_sum"] = rng.integers(0, 1 << 32, len(segs), dtype=np.uint64).astype(np.uint32)
    s["pre_sum"][:12] = 0
    arena = up(torch.from_numpy(host))  # no padding: the last chunk ends the allocation
    for comp in (0, 1):
        out = down(tc.batch_segments(arena, tc.descs_to_device(s), s.size, comp))
        exp = oracle.batch_segments(host, s, comp, nthreads=8)
        np.testing.assert_array_equal(out, exp)
    assert exp[10] == 0  # the 0xFFFF-folding range, complemented
    # peso form of the same ranges
    p = np.zeros(len(segs), tc.PESO_DTYPE)
    p["offset"], p["len"] = s["offset"], s["len"]
    p["src"] = rng.integers(0, 256, (len(segs), 4))
    p["dst"] = rng.integers(0, 256, (len(segs), 4))
    p["protocol"] = rng.choice([6, 17], len(segs))
    out = down(tc.batch_peso(arena, tc.descs_to_device(p), p.size))
    np.testing.assert_array_equal(out, oracle.batch_peso(host, p, nthreads=8))


def test_unsorted_overlapping_duplicate_descriptors(tc, torch, oracle):
    """Descriptors are independent reads: any order, overlaps, duplicates."""
    rng = np.random.default_rng(21)
    host = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    n = 30000
    p = np.zeros(n, tc.PESO_DTYPE)
    p["len"] = rng.integers(0, 4000, n)
    p["offset"] = rng.integers(0, host.size - 4000, n)
    p[n // 2:] = p[: n - n // 2]  # duplicates
    p["src"] = rng.integers(0, 256, (n, 4))
    p["dst"] = rng.integers(0, 256, (n, 4))
    p["protocol"] = rng.choice([6, 17, 1, 99], n)
    arena = up(torch.from_numpy(host))
    for mean in (0, 64, 1500, 70000):
        out = down(tc.batch_peso(arena, tc.descs_to_device(p), n, mean * n))
        np.testing.assert_array_equal(out, oracle.batch_peso(host, p, nthreads=8))


def test_hip_graph_capture_and_replay(tc, torch, oracle):
    """Batch calls allocate nothing and only enqueue: capturable in a hipGraph."""
    from tcp_amd import workload
    b = workload.make_batch("mtu", n=20000)
    arena, descs = workload.materialize(b)
    out = torch.empty(b.n, dtype=torch.uint16, device="cuda")
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        tc.batch_peso(arena, descs, b.n, b.total_bytes, out=out)
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    exp = oracle.batch_peso(down(arena), b.descs, nthreads=8)
    np.testing.assert_array_equal(down(out), exp)
    arena[: b.n * 1500].view(b.n, 1500)[:, 40] ^= 1  # new bytes, same graph
    g.replay()
    torch.cuda.synchronize()
    exp2 = oracle.batch_peso(down(arena), b.descs, nthreads=8)
    np.testing.assert_array_equal(down(out), exp2)
    assert (exp2 != exp).mean() > 0.99


def test_hip_graph_capture_tx_fill(tc, torch, oracle):
    """A tx fill large enough for the deferred form (>= 131,072 packets) takes
    the single-launch form under capture (no allocation inside a graph): the
    replayed graph fills the packets like the oracle, twice."""
    from tcp_amd import workload
    b = workload.make_batch("mixed_tx", n=140000)
    arena, descs = workload.materialize(b)
    unfilled = arena.clone()
    want = down(arena)
    oracle.batch_ipv4_tx_fill(want, b.descs, nthreads=8)
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        tc.batch_ipv4_tx_fill(arena, descs, b.n, b.total_bytes, want_flags=False)
    for _ in range(2):
        arena.copy_(unfilled)
        g.replay()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(down(arena), want)


def test_hip_graph_capture_tx_fill_scratch(tc, torch, oracle):
    """The deferred-store tx fill with caller scratch
    (tcsum_batch_ipv4_tx_fill_scratch) captured in a hipGraph: the replays
    fill the packets like the oracle and report the same values as the plain
    call; outside a graph it leaves the same bytes too."""
    from tcp_amd import workload
    b = workload.make_batch("mixed_tx", n=140000)
    arena, descs = workload.materialize(b)
    unfilled = arena.clone()
    want = down(arena)
    oracle.batch_ipv4_tx_fill(want, b.descs, nthreads=8)
    scratch = torch.empty(8 * b.n, dtype=torch.uint8, device="cuda")
    out = torch.empty(b.n, dtype=torch.uint32, device="cuda")
    ref_out = torch.empty_like(out)
    tc.batch_ipv4_tx_fill(arena, descs, b.n, b.total_bytes, out=ref_out, want_flags=False)
    torch.cuda.synchronize()
    assert np.array_equal(down(arena), want)
    arena.copy_(unfilled)
    tc.batch_ipv4_tx_fill(arena, descs, b.n, b.total_bytes, want_flags=False, scratch=scratch)  # no graph
    torch.cuda.synchronize()
    assert np.array_equal(down(arena), want)
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        tc.batch_ipv4_tx_fill(arena, descs, b.n, b.total_bytes, out=out, want_flags=False, scratch=scratch)
    for _ in range(2):
        arena.copy_(unfilled)
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(down(arena), want)
        assert torch.equal(out, ref_out)


def test_concurrent_streams(tc, torch, oracle):
    """Independent batches on independent streams do not interfere.  Outputs
    are allocated once up front: a tensor freed on one stream and reused by
    the caching allocator while another stream still writes it would race."""
    from tcp_amd import workload
    bs = [workload.make_batch(c, rank=r, n=n) for c, r, n in (("mtu", 0, 30000), ("mixed", 1, 8000), ("tso", 2, 64))]
    mats = [workload.materialize(b) for b in bs]
    outs = [torch.zeros(b.n, dtype=torch.uint16 if b.kind == "peso" else torch.uint32, device="cuda") for b in bs]
    streams = [torch.cuda.Stream() for _ in bs]
    torch.cuda.synchronize()
    for _ in range(3):
        for b, (arena, descs), o, st in zip(bs, mats, outs, streams):
            if b.kind == "peso":
                tc.batch_peso(arena, descs, b.n, b.total_bytes, out=o, stream=st)
            else:
                tc.batch_ipv4(arena, descs, b.n, b.total_bytes, out=o, want_flags=False, stream=st)
    torch.cuda.synchronize()
    for b, (arena, _), o in zip(bs, mats, outs):
        host = down(arena)
        exp = oracle.batch_peso(host, b.descs) if b.kind == "peso" else oracle.batch_ipv4(host, b.descs)[0]
        np.testing.assert_array_equal(down(o), exp)


def test_huge_batch_index_math(tc, torch, oracle, geometry):
    """More ranges than one launch may carry at one range per 1024-thread
    workgroup (2^22 - 1: the AQL packet counts work-items in 32 bits), so
    launch_segments cuts the batch into two launches; every result exact."""
    geometry(1024, 4)
    rng = np.random.default_rng(17)
    host = rng.integers(0, 256, 1 << 16, dtype=np.uint8)
    n = (1 << 22) + 1000
    s = np.zeros(n, tc.SEG_DTYPE)
    s["offset"] = rng.integers(0, (1 << 16) - 40, n)
    s["len"] = rng.integers(0, 33, n)
    s["pre_sum"] = rng.integers(0, 1 << 16, n)
    arena = up(torch.from_numpy(host))
    d = tc.descs_to_device(s)
    out = tc.batch_segments(arena, d, n, 1)
    exp = oracle.batch_segments(host, s, 1, nthreads=16)
    np.testing.assert_array_equal(down(out), exp)


def test_huge_ipv4_batch_index_math(tc, torch, oracle, geometry):
    """67M IPv4 packets at 64 lanes each (4 per workgroup): more than 2^24
    workgroups, so launch_ipv4 cuts the batch into two launches.  Sums, the tx
    fill (stores deferred: one scratch per launch) and rx verify give the
    oracle's values on a sample around the seam and spread over the batch."""
    geometry(64, 4)
    n, L = (1 << 26) + 1000, 28
    seam = ((1 << 24) - 1) * 4  # packets per launch at 64 lanes (kMaxBlocks)
    rng = np.random.default_rng(23)
    host = rng.integers(0, 256, (n, L), dtype=np.uint8)
    host[:, 0], host[:, 1], host[:, 2], host[:, 3] = 0x45, 0, 0, L  # IHL 5, total_len 28
    host[:, 6] &= 0x40  # DF at most: no fragments
    host[:, 7] = 0
    host[:, 9] = np.where(rng.integers(0, 2, n) == 0, 17, 1)  # UDP or ICMP
    pk = np.zeros(n, tc.PKT_DTYPE)
    pk["offset"] = np.arange(n, dtype=np.uint64) * np.uint64(L)
    pk["len"] = L
    idx = np.unique(np.concatenate([np.arange(2000), np.arange(seam - 3000, n), rng.choice(n, 50000)]))
    sample = np.ascontiguousarray(host[idx]).reshape(-1)
    spk = np.zeros(idx.size, tc.PKT_DTYPE)
    spk["offset"] = np.arange(idx.size, dtype=np.uint64) * np.uint64(L)
    spk["len"] = L
    arena = up(torch.from_numpy(host.reshape(-1)))
    del host
    d = tc.descs_to_device(pk)
    tidx = up(torch.from_numpy(idx))

    out, flags = tc.batch_ipv4(arena, d, n, n * L)
    eo, ef = oracle.batch_ipv4(sample, spk)
    np.testing.assert_array_equal(down(out.view(torch.int32)[tidx]).view(np.uint32), eo)
    np.testing.assert_array_equal(down(flags[tidx]), ef)
    del out, flags

    tflags = tc.batch_ipv4_tx_fill(arena, d, n, n * L)  # 28-B packets: the stores in the kernel
    efl = oracle.batch_ipv4_tx_fill(sample, spk)  # sample is filled in place
    np.testing.assert_array_equal(down(tflags[tidx]), efl)
    got = down(arena.view(n, L)[tidx]).reshape(-1)
    np.testing.assert_array_equal(got, sample)
    with tc.debug(tx_split=1):  # and deferred to k_tx_scatter (idempotent: the fields read as zero)
        tflags = tc.batch_ipv4_tx_fill(arena, d, n, n * L)
    np.testing.assert_array_equal(down(tflags[tidx]), efl)
    np.testing.assert_array_equal(down(arena.view(n, L)[tidx]).reshape(-1), sample)

    verdict, vflags = tc.batch_ipv4_rx_verify(arena, d, n, n * L)
    ev, evf = oracle.batch_ipv4_rx_verify(sample, spk)
    np.testing.assert_array_equal(down(verdict[tidx]), ev)
    np.testing.assert_array_equal(down(vflags[tidx]), evf)


@pytest.mark.parametrize("order,chunk_mb", [("permuted", None), ("offset", None), ("offset", "1")])
def test_host_batch_end_to_end(tc, oracle, knobs, order, chunk_mb):
    """Pageable host arena -> H2D -> kernel -> D2H matches the device-resident
    path: descriptors in any order (one span copy) and in offset order (the
    chunk pipeline; 1 MiB chunks = one per 4096-segment block, 11 chunks)."""
    from tcp_amd import workload
    if chunk_mb:
        knobs(e2e_chunk_mb=int(chunk_mb))
    b = workload.make_batch("mtu", n=43000)
    host = oracle.synth_fill(b.byte_base, b.alloc_bytes, b.seed)
    rng = np.random.default_rng(3)
    d = b.descs[rng.permutation(b.n)] if order == "permuted" else b.descs
    out = tc.host_batch_peso(host, d)
    np.testing.assert_array_equal(out, oracle.batch_peso(host, d, nthreads=8))


@pytest.mark.parametrize("order", ["offset", "permuted"])
def test_host_batch_pageable_staging(tc, oracle, order):
    """A pageable arena crosses through the context's three 32-MiB pinned
    slots -- 150 MB, so every slot is refilled after its copy-done event.
    (The runtime's own pageable copy, debug knob page_stage = 0, is not run
    here: DESIGN.md §4.)"""
    from tcp_amd import workload
    b = workload.make_batch("mtu", n=100000)
    host = oracle.synth_fill(b.byte_base, b.alloc_bytes, b.seed)
    d = b.descs[np.random.default_rng(8).permutation(b.n)] if order == "permuted" else b.descs
    out = tc.host_batch_peso(host, d)
    np.testing.assert_array_equal(out, oracle.batch_peso(host, d, nthreads=8))


@pytest.mark.parametrize("case", ["late_low", "rest_empty", "lead_sparse", "chunks"])
def test_host_batch_lead_and_rest(tc, oracle, knobs, case):
    """The host batch's lead (its first 64 MiB of segments, copied before the
    rest of the descriptors are read, into a buffer of its own when dense)
    and the rest: a later segment back inside / below the lead's span, a rest
    of empty segments, a sparse lead (no early copy), several rest chunks."""
    from tcp_amd import workload
    b = workload.make_batch("mtu", n=60000)  # 90 MB: a 64-MiB lead + a rest
    host = oracle.synth_fill(b.byte_base, b.alloc_bytes, b.seed)
    d = b.descs.copy()
    if case == "late_low":
        d[-100:]["offset"] = d[:100]["offset"][::-1] + 3  # back inside the lead's bytes
        d[-100:]["len"] = 1400
    elif case == "rest_empty":
        d[50000:]["len"] = 0
    elif case == "lead_sparse":
        d = d[::2].copy()  # every other 1500-B slot: the lead's span is 2x its bytes
    else:
        knobs(e2e_chunk_mb=8)
    out = tc.host_batch_peso(host, d)
    np.testing.assert_array_equal(out, oracle.batch_peso(host, d, nthreads=8))


def test_host_batch_long_segments(tc, oracle):
    """The host batch's 16-byte descriptors carry the pseudo-header folded on
    the host: segments of 64 KiB and longer (the length word is (u16)len,
    tools.c:69 -- 65,536 B gives 0), odd offsets, empty ones, every protocol
    byte value."""
    rng = np.random.default_rng(91)
    lens = np.array([65535, 65536, 65537, 70000, 131072, 0, 1, 2, 9000, 65534] * 8)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]) + rng.integers(0, 2, lens.size).cumsum()
    host = rng.integers(0, 256, int(offs[-1] + lens[-1] + 64), dtype=np.uint8)
    p = np.zeros(lens.size, tc.PESO_DTYPE)
    p["offset"], p["len"] = offs, lens
    p["src"] = rng.integers(0, 256, (lens.size, 4))
    p["dst"] = rng.integers(0, 256, (lens.size, 4))
    p["protocol"] = rng.integers(0, 256, lens.size)
    out = tc.host_batch_peso(host, p)
    np.testing.assert_array_equal(out, oracle.batch_peso(host, p, nthreads=4))


@pytest.mark.parametrize("shift", [0, 7])
def test_host_batch_pinned(tc, oracle, shift):
    """A pinned arena (tcsum_host_alloc), ragged segments in any order, at an
    odd arena base too: same results as the oracle."""
    import ctypes
    from tcp_amd import _lib, workload
    b = workload.make_batch("mtu", n=20000)
    L = _lib.lib()
    nbytes = b.alloc_bytes + shift
    p = L.tcsum_host_alloc(nbytes)
    assert p
    try:
        host = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p))[shift:]
        host[:] = oracle.synth_fill(b.byte_base, b.alloc_bytes, b.seed)
        rng = np.random.default_rng(5)
        segs = np.zeros(b.n, tc.PESO_DTYPE)
        segs["offset"] = b.descs["offset"]
        segs["len"] = rng.integers(0, 1501, b.n)  # ragged, inside each 1500-B slot
        segs["src"] = rng.integers(0, 256, (b.n, 4))
        segs["dst"] = rng.integers(0, 256, (b.n, 4))
        segs["protocol"] = rng.choice([6, 17], b.n)
        segs = segs[rng.permutation(b.n)]
        out = tc.host_batch_peso(host, segs)
        np.testing.assert_array_equal(out, oracle.batch_peso(np.array(host), segs, nthreads=8))
    finally:
        L.tcsum_host_free(p)


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0, 0, 0]])
def test_host_batch_multi_device(tc, oracle, devices):
    """tcsum_host_batch_peso_multi: byte-balanced shards over a device list
    (one GPU here, listed repeatedly: every shard boundary and the span-only
    device arena are exercised), ragged segments in any order, results in
    segment order; also fewer segments than devices."""
    rng = np.random.default_rng(31)
    host = rng.integers(0, 256, 12 << 20, dtype=np.uint8)
    n = 30000
    p = np.zeros(n, tc.PESO_DTYPE)
    p["len"] = rng.integers(0, 9000, n)
    p["offset"] = rng.integers(0, host.size - 9000, n)
    p["src"] = rng.integers(0, 256, (n, 4))
    p["dst"] = rng.integers(0, 256, (n, 4))
    p["protocol"] = rng.choice([6, 17], n)
    out = tc.host_batch_peso_multi(host, p, devices)
    np.testing.assert_array_equal(out, oracle.batch_peso(host, p, nthreads=8))
    # every shard recorded: its device, its contiguous descriptors, its bytes and time
    sh = tc.last_shards()
    assert [s["device"] for s in sh] == list(devices) and all(s["rc"] == 0 for s in sh)
    assert [s["first"] for s in sh] == list(np.cumsum([0] + [s["count"] for s in sh[:-1]]))
    assert sum(s["count"] for s in sh) == n and sum(s["bytes"] for s in sh) == int(p["len"].sum())
    assert all(s["ms"] > 0 for s in sh if s["count"])
    few = p[:2].copy()
    few["offset"] = [host.size - 100, 5]  # the span is not in offset order
    few["len"] = [100, 51]
    np.testing.assert_array_equal(tc.host_batch_peso_multi(host, few, devices),
                                  oracle.batch_peso(host, few, nthreads=1))


@pytest.mark.parametrize("devices", [[0, 0, 0], [0] * 7])
def test_host_batch_multi_device_many_blocks(tc, oracle, devices):
    """The multi-device shard cuts over many 64K-descriptor blocks (the cut
    search runs per block, in parallel): 400,000 ragged segments in offset
    order, some empty runs, results in segment order."""
    rng = np.random.default_rng(77)
    n = 400000
    lens = rng.integers(0, 1501, n)
    lens[100000:130000] = 0  # an empty run: quantiles fall around it
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]) + 3
    host = rng.integers(0, 256, int(offs[-1] + lens[-1] + 64), dtype=np.uint8)
    p = np.zeros(n, tc.PESO_DTYPE)
    p["offset"], p["len"] = offs, lens
    p["src"] = rng.integers(0, 256, (n, 4))
    p["dst"] = rng.integers(0, 256, (n, 4))
    p["protocol"] = rng.choice([6, 17], n)
    out = tc.host_batch_peso_multi(host, p, devices)
    np.testing.assert_array_equal(out, oracle.batch_peso(host, p, nthreads=8))


# --------------------------------------------------- full BASELINE sizes

def test_full_mtu_batch_exact(tc, torch, oracle):
    """configs[1] at full size (1M x 1500 B): every result checked."""
    b, arena, out = run_config(tc, torch, "mtu", None)
    exp = oracle.batch_peso(down(arena), b.descs, nthreads=16)
    np.testing.assert_array_equal(down(out), exp)


def test_full_mixed_batch_exact(tc, torch, oracle):
    """configs[3] at full size (1M packets, ~4.4 GiB): every result checked."""
    b, arena, out = run_config(tc, torch, "mixed", None)
    exp, fl = oracle.batch_ipv4(down(arena), b.descs, nthreads=16)
    np.testing.assert_array_equal(down(out), exp)


def test_full_tso_batch_properties(tc, torch, oracle):
    """configs[2] at full size (256K x 64 KiB = 16 GiB): every segment exact,
    run-to-run determinism, geometry invariance, and the RFC 1624 incremental
    update on every segment (changing one 16-bit word m -> m' turns checksum
    HC into ~(~HC + ~m + m'))."""
    from tcp_amd import workload
    b = workload.make_batch("tso")
    arena, descs = workload.materialize(b)
    out1 = tc.batch_peso(arena, descs, b.n, b.total_bytes)
    out2 = tc.batch_peso(arena, descs, b.n, b.total_bytes)
    torch.cuda.synchronize()
    hc = down(out1)
    np.testing.assert_array_equal(hc, down(out2))
    with tc.debug(lanes=256, loads=16):  # k_segments_wg instead of k_segments_wgx
        out3 = tc.batch_peso(arena, descs, b.n, b.total_bytes)
    np.testing.assert_array_equal(hc, down(out3))
    # every segment exact: the 16 GiB arena copied to the host once, the
    # oracle over all 262,144 segments on 16 threads
    host = down(arena)
    np.testing.assert_array_equal(hc, oracle.batch_peso(host, b.descs, nthreads=16))
    del host
    # sampled exact parity through the single-segment oracle entry point
    rng = np.random.default_rng(11)
    idx = np.sort(rng.choice(b.n, 512, replace=False))
    for i in idx:
        o, L = int(b.descs["offset"][i]), int(b.descs["len"][i])
        seg = down(arena[o: o + L])
        assert hc[i] == oracle.checksum_peso(seg, b.descs["dst"][i], b.descs["src"][i], 6)
    # incremental update: rewrite the word at offset 100 of every segment
    words = arena[: b.n * 65536].view(b.n, 65536)
    old = down(words[:, 100:102]).copy().view("<u2").reshape(-1).astype(np.uint32)
    new_bytes = up(torch.from_numpy(rng.integers(0, 256, (b.n, 2), dtype=np.uint8)))
    words[:, 100:102] = new_bytes
    new = down(new_bytes).copy().view("<u2").reshape(-1).astype(np.uint32)
    out4 = down(tc.batch_peso(arena, descs, b.n, b.total_bytes)).astype(np.uint32)
    s = (~hc.astype(np.uint32) & 0xFFFF) + (~old & 0xFFFF) + new
    s = (s & 0xFFFF) + (s >> 16)
    s = (s & 0xFFFF) + (s >> 16)
    np.testing.assert_array_equal(out4, ~s & 0xFFFF)


# --------------------------------------------------- seeded fuzz

def _fuzz_arena(rng, size):
    host = rng.integers(0, 256, size, dtype=np.uint8)
    for _ in range(40):  # long runs of 0x00 / 0xFF (fold edge cases)
        a = int(rng.integers(0, size - 5000))
        host[a: a + int(rng.integers(1, 5000))] = rng.choice([0, 0xFF])
    return host


def _fuzz_lens(rng, n, hi):
    kind = rng.integers(0, 3, n)
    return np.where(kind == 0, rng.integers(0, 65, n),
                    np.where(kind == 1, rng.integers(0, 2048, n), rng.integers(0, hi, n)))


@pytest.mark.parametrize("seed", range(12))
def test_fuzz_vs_oracle(tc, torch, oracle, geometry, seed):
    """Random geometry, ragged ranges at random offsets over data with long
    0x00 / 0xFF runs; then semi-valid IPv4 packets (random version, IHL,
    total length, fragment bits, protocol, stored checksums) through sums,
    tx fill and rx verify.  Everything must equal the oracle."""
    rng = np.random.default_rng(9000 + seed)
    size = 8 << 20
    host = _fuzz_arena(rng, size)
    arena = up(torch.from_numpy(host))
    geometry(*GEOMS_SEG[int(rng.integers(0, len(GEOMS_SEG)))])
    n = 4000
    lens = _fuzz_lens(rng, n, 70000)
    s = np.zeros(n, tc.SEG_DTYPE)
    s["len"] = lens
    s["offset"] = rng.integers(0, size - lens)
    s["pre_sum"] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    comp = int(rng.integers(0, 2))
    out = down(tc.batch_segments(arena, tc.descs_to_device(s), n, comp))
    np.testing.assert_array_equal(out, oracle.batch_segments(host, s, comp, nthreads=8))
    p = np.zeros(n, tc.PESO_DTYPE)
    p["offset"], p["len"] = s["offset"], s["len"]
    p["src"] = rng.integers(0, 256, (n, 4))
    p["dst"] = rng.integers(0, 256, (n, 4))
    p["protocol"] = rng.choice([6, 17], n)
    out = down(tc.batch_peso(arena, tc.descs_to_device(p), n))
    np.testing.assert_array_equal(out, oracle.batch_peso(host, p, nthreads=8))

    # IPv4 packets packed with random gaps; headers mostly plausible
    geometry(*GEOMS_IP[int(rng.integers(0, len(GEOMS_IP)))])
    m = 1500
    plen = _fuzz_lens(rng, m, 9001)
    gaps = rng.integers(0, 40, m)
    offs = np.cumsum(np.concatenate([[int(rng.integers(0, 16))], (plen + gaps)[:-1]]))
    assert offs[-1] + plen[-1] < size
    pk = np.zeros(m, tc.PKT_DTYPE)
    pk["offset"], pk["len"] = offs, plen
    ip = host.copy()
    for o, ln in zip(offs.tolist(), plen.tolist()):
        if ln < 20:
            continue
        h = ip[o: o + 20]
        h[0] = 0x45 if rng.random() < 0.85 else int(rng.integers(0, 256))
        tl = ln if rng.random() < 0.8 else int(rng.integers(0, 70000)) & 0xFFFF
        h[2], h[3] = tl >> 8, tl & 0xFF
        if rng.random() < 0.85:
            h[6], h[7] = 0, 0  # not a fragment
        h[9] = int(rng.choice([6, 17, 1, 99]))
        if rng.random() < 0.2:
            h[10], h[11] = 0, 0  # stored header checksum 0: rx skips it
        if ln >= 40 and rng.random() < 0.2:
            ip[o + 20 + 16: o + 20 + 18] = 0  # TCP checksum field zero (rx skip rule)
            ip[o + 20 + 6: o + 20 + 8] = 0    # UDP checksum field zero
    d_ip = up(torch.from_numpy(ip))
    d_pk = tc.descs_to_device(pk)
    out, fl = tc.batch_ipv4(d_ip, d_pk, m)
    exp, efl = oracle.batch_ipv4(ip, pk, nthreads=8)
    np.testing.assert_array_equal(down(out), exp)
    np.testing.assert_array_equal(down(fl), efl)
    verdict, vfl = tc.batch_ipv4_rx_verify(d_ip, d_pk, m)
    ev, evfl = oracle.batch_ipv4_rx_verify(ip, pk, nthreads=8)
    np.testing.assert_array_equal(down(verdict), ev)
    tfl = tc.batch_ipv4_tx_fill(d_ip, d_pk, m)
    efl2 = oracle.batch_ipv4_tx_fill(ip, pk, nthreads=8)  # ip is filled in place
    np.testing.assert_array_equal(down(tfl), efl2)
    np.testing.assert_array_equal(down(d_ip), ip)
    # and verify what was filled: well-formed packets now pass
    verdict, _ = tc.batch_ipv4_rx_verify(d_ip, d_pk, m)
    ev, _ = oracle.batch_ipv4_rx_verify(ip, pk, nthreads=8)
    np.testing.assert_array_equal(down(verdict), ev)
    assert (ev == 0).sum() > m // 4


@pytest.mark.parametrize("config", ["mtu", "tso", "mixed", "mixed_rx"])
def test_measurement_probes_leave_arena_and_sink_alone(torch, tc, config):
    """bench.py's achievable-side probes (tcsum_probe_read / _tile /
    _segments / _ipv4) read the batch and write nothing but a 2^-32 sink: the arena is
    unchanged, the sink still 0, and every geometry pick_geometry returns for
    a batch has a probe_segments / probe_ipv4 instance."""
    from tcp_amd import workload
    n = {"mtu": 20000, "tso": 64, "mixed": 4000, "mixed_rx": 4000}[config]
    b = workload.make_batch(config, n=n)
    arena, descs = workload.materialize(b)
    before = arena.clone()
    sink = torch.zeros(1, dtype=torch.uint32, device=arena.device)
    tc.probe_read(arena, b.arena_bytes, sink)
    g, u = tc.pick_geometry(b.total_bytes // b.n)
    if g <= 256:  # the tile probe has the <= 256-lane shapes (bench.py skips it otherwise)
        tc.probe_tile(arena, b.arena_bytes, g, u, sink)
    if b.kind == "peso":
        tc.probe_segments(arena, descs, b.n, b.total_bytes, sink)
    else:
        tc.probe_ipv4(arena, descs, b.n, b.total_bytes, rx=b.op == "rx", sink=sink)
    torch.cuda.synchronize()
    assert int(sink.item()) == 0
    assert torch.equal(arena, before)


@pytest.mark.parametrize("g,u", [(4, 1), (8, 4), (16, 6), (32, 6), (256, 16), (1024, 4)])
def test_ragged_batch_sizes_write_only_their_results(tc, torch, oracle, geometry, g, u):
    """Batch sizes that leave the last workgroup partly empty (k_segments
    stores a workgroup's results from its last wave, k_ipv4 per packet): every
    result equals the oracle's and nothing past out[n) is written."""
    rng = np.random.default_rng(77)
    host = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    arena = up(torch.from_numpy(host))
    geometry(g, u)
    for n in (1, 2, 3, 15, 17, 63, 65, 1001):
        p = np.zeros(n, tc.PESO_DTYPE)
        p["len"] = rng.integers(1, 3000, n)
        p["offset"] = rng.integers(0, host.size - 3000, n)
        p["src"] = rng.integers(0, 256, (n, 4))
        p["dst"] = rng.integers(0, 256, (n, 4))
        p["protocol"] = rng.choice([6, 17], n)
        out = torch.full((n + 300,), 0xABCD, dtype=torch.int32, device="cuda").view(torch.uint16)
        tc.batch_peso(arena, tc.descs_to_device(p), n, int(p["len"].sum()), out=out)
        got = down(out)
        np.testing.assert_array_equal(got[:n], oracle.batch_peso(host, p, nthreads=8))
        sentinel = np.full(n + 300, 0xABCD, np.int32).view(np.uint16)  # int32 fill seen as u16 pairs
        np.testing.assert_array_equal(got[n:], sentinel[n:])
