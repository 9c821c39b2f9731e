"""Python face of the engine: the reference's checksum interface, plus batches.

Same names, argument meanings and results as the reference:

    checksum16(offset, buf, len, pre_sum, complement)   net/src/tools.c:24-54
    checksum_peso(buf, dest, src, protocol)              net/src/tools.c:56-75
    pktbuf_checksum16(buf, len, pre_sum, complement)     net/src/pktbuf.c:646-670

each a thin call into libtcsum.so, where the sum runs on the GPU.  The batch
forms take device (torch CUDA) tensors: a uint8 arena and a descriptor array
laid out as include/tcsum.h's structs (SEG_DTYPE / PESO_DTYPE / PKT_DTYPE).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .pktbuf import IpAddr, PktBuf

SEG_DTYPE = np.dtype([("offset", "<u8"), ("len", "<u4"), ("pre_sum", "<u4")])
PESO_DTYPE = np.dtype([("offset", "<u8"), ("len", "<u4"), ("src", "u1", 4),
                       ("dst", "u1", 4), ("protocol", "u1"), ("rsv", "u1", 3)])
PKT_DTYPE = np.dtype([("offset", "<u8"), ("len", "<u4"), ("rsv", "<u4")])

PKT_BAD_VERSION, PKT_BAD_HDRLEN, PKT_BAD_TOTLEN, PKT_PROTO_OTHER, PKT_SHORT = 1, 2, 4, 8, 16
PKT_FRAGMENT, PKT_L4_SHORT = 32, 64


# ------------------------------------------------------------- drop-in trio

def checksum16(offset: int, buf, length: int, pre_sum: int, complement: int) -> int:
    """tools.c:24-54 on a host buffer (bytes-like or numpy)."""
    if isinstance(buf, np.ndarray):
        a = np.ascontiguousarray(buf.reshape(-1).view(np.uint8))
        ptr = a.ctypes.data if a.size else None
        assert length <= a.size
        return _lib.lib().checksum16(offset, ptr, length, pre_sum & 0xFFFFFFFF, complement)
    b = bytes(buf)
    assert length <= len(b)
    cbuf = ctypes.create_string_buffer(b, max(1, len(b)))
    return _lib.lib().checksum16(offset, ctypes.addressof(cbuf), length, pre_sum & 0xFFFFFFFF, complement)


def pktbuf_checksum16(buf: PktBuf, length: int, pre_sum: int, complement: int) -> int:
    """pktbuf.c:646-670: from the cursor; advances it by `length`."""
    return _lib.lib().pktbuf_checksum16(buf.ptr, length, pre_sum, complement)


def checksum_peso(buf: PktBuf, dest: IpAddr, src: IpAddr, protocol: int) -> int:
    """tools.c:56-75: resets the cursor, leaves it at the end."""
    return _lib.lib().checksum_peso(buf.ptr, ctypes.addressof(dest), ctypes.addressof(src), protocol)


# ------------------------------------------------------------------ batches

def _torch():
    import torch
    return torch


def descs_to_device(descs: np.ndarray, device="cuda"):
    """Copy a structured descriptor array to the device as raw bytes, through
    pinned host memory: the runtime's own pageable host-to-device path is the
    one three GPU suites stopped on."""
    torch = _torch()
    raw = np.ascontiguousarray(descs).view(np.uint8)
    return torch.from_numpy(raw.copy()).pin_memory().to(device)


_HOST_CHUNK = 64 << 20


def to_host_tensor(t):
    """A device tensor's values in host memory, copied by the GPU only into
    pinned memory: the runtime's pageable device-to-host path is, with the
    host-to-device one, where the round-5 GPU suites stopped.
    Up to 64 MiB: one pinned tensor; larger: chunk by chunk through a 64-MiB
    pinned bounce buffer into a pageable tensor (a power-of-two pinned block
    per multi-GB result would pin twice its size).  Synchronous, like
    `.cpu()`; a host tensor is returned as it is."""
    torch = _torch()
    if t.device.type != "cuda":
        return t
    src = t.contiguous().reshape(-1)
    per = max(1, _HOST_CHUNK // src.element_size())
    if src.numel() <= per:
        h = torch.empty(src.numel(), dtype=src.dtype, pin_memory=True)
        h.copy_(src)
        return h.reshape(t.shape)
    out = torch.empty(src.numel(), dtype=src.dtype)
    bounce = torch.empty(per, dtype=src.dtype, pin_memory=True)
    for o in range(0, src.numel(), per):
        k = min(per, src.numel() - o)
        bounce[:k].copy_(src[o:o + k])
        out[o:o + k].copy_(bounce[:k])
    return out.reshape(t.shape)


def to_host(t) -> np.ndarray:
    """to_host_tensor(t) as a numpy array."""
    return to_host_tensor(t).numpy()


def _stream_ptr(stream) -> int | None:
    torch = _torch()
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


LAYOUT_UNKNOWN, LAYOUT_ORDERED, LAYOUT_SHUFFLED = 0, 1, 2
OP_SEGMENTS, OP_SEGMENTS_COMP, OP_PESO, OP_IPV4, OP_IPV4_TX_FILL, OP_IPV4_TX_OFFLOAD, OP_IPV4_RX_VERIFY = range(7)


class Hint(ctypes.Structure):
    """tcsum_hint_t: the batch's byte count and what the caller knows of its layout."""
    _fields_ = [("total_bytes", ctypes.c_uint64), ("layout", ctypes.c_uint32), ("rsv", ctypes.c_uint32)]


def batch(op: int, arena, descs, n: int, out=None, flags=None, verdict=None, total_bytes: int = 0,
          layout: int = LAYOUT_UNKNOWN, stream=None):
    """tcsum_batch: any device-resident batch with a layout hint (device
    tensors; out / flags / verdict as the op needs them, allocated when None)."""
    torch = _torch()
    dev = arena.device
    if out is None and op != OP_IPV4_RX_VERIFY and op != OP_IPV4_TX_FILL:
        out = torch.empty(n, dtype=torch.uint16 if op <= OP_PESO else torch.uint32, device=dev)
    if flags is None and op == OP_IPV4_TX_OFFLOAD:
        flags = torch.empty(n, dtype=torch.uint8, device=dev)
    if verdict is None and op == OP_IPV4_RX_VERIFY:
        verdict = torch.empty(n, dtype=torch.int8, device=dev)
    h = Hint(total_bytes, layout, 0)
    ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    rc = _lib.lib().tcsum_batch(op, arena.data_ptr(), descs.data_ptr(), n, ptr(out), ptr(flags), ptr(verdict),
                                ctypes.byref(h), _stream_ptr(stream))
    _lib.check(rc, "tcsum_batch")
    return out, flags, verdict


def batch_segments(arena, segs, n: int, complement: int, total_bytes: int = 0, out=None, stream=None):
    """out[i] = pktbuf_checksum16 over each tcsum_seg_t (device tensors)."""
    torch = _torch()
    if out is None:
        out = torch.empty(n, dtype=torch.uint16, device=arena.device)
    rc = _lib.lib().tcsum_batch_segments(arena.data_ptr(), segs.data_ptr(), n, out.data_ptr(),
                                         complement, total_bytes, _stream_ptr(stream))
    _lib.check(rc, "tcsum_batch_segments")
    return out


def batch_peso(arena, segs, n: int, total_bytes: int = 0, out=None, stream=None):
    """out[i] = checksum_peso over each tcsum_peso_t (device tensors)."""
    torch = _torch()
    if out is None:
        out = torch.empty(n, dtype=torch.uint16, device=arena.device)
    rc = _lib.lib().tcsum_batch_peso(arena.data_ptr(), segs.data_ptr(), n, out.data_ptr(), total_bytes,
                                     _stream_ptr(stream))
    _lib.check(rc, "tcsum_batch_peso")
    return out


def batch_ipv4(arena, pkts, n: int, total_bytes: int = 0, out=None, flags=None, want_flags=True, stream=None):
    """(out, flags): out[i] = ip | l4 << 16 for each tcsum_pkt_t (device tensors)."""
    torch = _torch()
    if out is None:
        out = torch.empty(n, dtype=torch.uint32, device=arena.device)
    if flags is None and want_flags:
        flags = torch.empty(n, dtype=torch.uint8, device=arena.device)
    rc = _lib.lib().tcsum_batch_ipv4(arena.data_ptr(), pkts.data_ptr(), n, out.data_ptr(),
                                     flags.data_ptr() if flags is not None else None, total_bytes,
                                     _stream_ptr(stream))
    _lib.check(rc, "tcsum_batch_ipv4")
    return out, flags


def batch_ipv4_tx_fill(arena, pkts, n: int, total_bytes: int = 0, out=None, flags=None, want_flags=True,
                       stream=None, scratch=None):
    """Write the IPv4 / TCP / UDP / ICMP checksums into the packets in place.
    scratch: a device tensor of >= 8*n bytes the caller owns
    (tcsum_batch_ipv4_tx_fill_scratch: the deferred-store form with no
    allocation, capturable in a hipGraph)."""
    torch = _torch()
    if flags is None and want_flags:
        flags = torch.empty(n, dtype=torch.uint8, device=arena.device)
    o = out.data_ptr() if out is not None else None
    f = flags.data_ptr() if flags is not None else None
    if scratch is None:
        rc = _lib.lib().tcsum_batch_ipv4_tx_fill(arena.data_ptr(), pkts.data_ptr(), n, o, f, total_bytes,
                                                 _stream_ptr(stream))
    else:
        rc = _lib.lib().tcsum_batch_ipv4_tx_fill_scratch(arena.data_ptr(), pkts.data_ptr(), n, o, f,
                                                         scratch.data_ptr(),
                                                         scratch.numel() * scratch.element_size(), total_bytes,
                                                         _stream_ptr(stream))
    _lib.check(rc, "tcsum_batch_ipv4_tx_fill")
    return flags


def batch_ipv4_rx_verify(arena, pkts, n: int, total_bytes: int = 0, verdict=None, out=None, flags=None,
                         want_flags=True, stream=None):
    """(verdict int8 net_err_t, flags) per packet, as the stack's rx gates decide."""
    torch = _torch()
    if verdict is None:
        verdict = torch.empty(n, dtype=torch.int8, device=arena.device)
    if flags is None and want_flags:
        flags = torch.empty(n, dtype=torch.uint8, device=arena.device)
    rc = _lib.lib().tcsum_batch_ipv4_rx_verify(arena.data_ptr(), pkts.data_ptr(), n, verdict.data_ptr(),
                                               out.data_ptr() if out is not None else None,
                                               flags.data_ptr() if flags is not None else None, total_bytes,
                                               _stream_ptr(stream))
    _lib.check(rc, "tcsum_batch_ipv4_rx_verify")
    return verdict, flags


def host_batch_peso(host_arena: np.ndarray, segs: np.ndarray, device: int = 0) -> np.ndarray:
    """End-to-end: host arena -> H2D -> kernel -> D2H (tcsum_host_batch_peso)."""
    assert segs.dtype == PESO_DTYPE
    segs = np.ascontiguousarray(segs)  # held for the call: a temporary's buffer could be freed before it
    out = np.zeros(segs.size, np.uint16)
    rc = _lib.lib().tcsum_host_batch_peso(device, host_arena.ctypes.data, host_arena.nbytes,
                                          segs.ctypes.data, segs.size, out.ctypes.data)
    _lib.check(rc, "tcsum_host_batch_peso")
    return out


def host_batch_peso_multi(host_arena: np.ndarray, segs: np.ndarray, devices) -> np.ndarray:
    """tcsum_host_batch_peso_multi: one host batch sharded by bytes over `devices`."""
    assert segs.dtype == PESO_DTYPE
    devs = np.ascontiguousarray(np.asarray(list(devices), dtype=np.int32))
    segs = np.ascontiguousarray(segs)
    out = np.zeros(segs.size, np.uint16)
    rc = _lib.lib().tcsum_host_batch_peso_multi(devs.ctypes.data, devs.size, host_arena.ctypes.data,
                                                host_arena.nbytes, segs.ctypes.data,
                                                segs.size, out.ctypes.data)
    _lib.check(rc, "tcsum_host_batch_peso_multi")
    return out


class HostArena:
    """Pinned host memory from tcsum_host_alloc (the plat/ pinned pool), viewed
    as a numpy u8 array; the kernels read and write it in place."""

    def __init__(self, nbytes: int):
        self.nbytes = int(nbytes)
        self._ptr = _lib.lib().tcsum_host_alloc(max(self.nbytes, 1))
        if not self._ptr:
            raise MemoryError(f"tcsum_host_alloc({nbytes}) failed")
        buf = (ctypes.c_uint8 * max(self.nbytes, 1)).from_address(self._ptr)
        self.array = np.ctypeslib.as_array(buf)[: self.nbytes]

    def free(self):
        if self._ptr:
            self.array = None
            _lib.lib().tcsum_host_free(self._ptr)
            self._ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def host_register(arr: np.ndarray) -> None:
    """Pin an existing u8 array in place (tcsum_host_register)."""
    _lib.check(_lib.lib().tcsum_host_register(arr.ctypes.data, arr.nbytes), "tcsum_host_register")


def host_unregister(arr: np.ndarray) -> None:
    _lib.check(_lib.lib().tcsum_host_unregister(arr.ctypes.data), "tcsum_host_unregister")


def _host_arena_args(host_arena):
    arr = host_arena.array if isinstance(host_arena, HostArena) else host_arena
    assert arr.dtype == np.uint8 and arr.flags["C_CONTIGUOUS"]
    return arr.ctypes.data, arr.nbytes


def _devices(devices):
    d = np.ascontiguousarray(np.asarray(list(devices), dtype=np.int32))
    return d.ctypes.data, d.size, d


def host_batch_ipv4(host_arena, pkts: np.ndarray, device: int = 0, devices=None):
    """(out u32 = ip | l4 << 16, flags) for packets in host memory
    (tcsum_host_batch_ipv4; with `devices`, sharded by bytes over those GPUs:
    tcsum_host_batch_ipv4_multi)."""
    assert pkts.dtype == PKT_DTYPE
    pkts = np.ascontiguousarray(pkts)
    out = np.zeros(pkts.size, np.uint32)
    flags = np.zeros(pkts.size, np.uint8)
    p, nb = _host_arena_args(host_arena)
    if devices is None:
        rc = _lib.lib().tcsum_host_batch_ipv4(device, p, nb, pkts.ctypes.data, pkts.size, out.ctypes.data,
                                              flags.ctypes.data)
    else:
        dp, nd, _keep = _devices(devices)
        rc = _lib.lib().tcsum_host_batch_ipv4_multi(dp, nd, p, nb, pkts.ctypes.data, pkts.size, out.ctypes.data,
                                                    flags.ctypes.data)
    _lib.check(rc, "tcsum_host_batch_ipv4")
    return out, flags


def host_batch_ipv4_tx_fill(host_arena, pkts: np.ndarray, device: int = 0, devices=None):
    """Fill the checksum fields of packets in host memory in place; returns
    flags (with `devices`: tcsum_host_batch_ipv4_tx_fill_multi)."""
    assert pkts.dtype == PKT_DTYPE
    pkts = np.ascontiguousarray(pkts)
    flags = np.zeros(pkts.size, np.uint8)
    p, nb = _host_arena_args(host_arena)
    if devices is None:
        rc = _lib.lib().tcsum_host_batch_ipv4_tx_fill(device, p, nb, pkts.ctypes.data, pkts.size, None,
                                                      flags.ctypes.data)
    else:
        dp, nd, _keep = _devices(devices)
        rc = _lib.lib().tcsum_host_batch_ipv4_tx_fill_multi(dp, nd, p, nb, pkts.ctypes.data, pkts.size, None,
                                                            flags.ctypes.data)
    _lib.check(rc, "tcsum_host_batch_ipv4_tx_fill")
    return flags


def batch_ipv4_tx_offload(arena, pkts, n: int, total_bytes: int = 0, out=None, flags=None, stream=None):
    """(out u32 = ip | l4 << 16, flags): the values batch_ipv4_tx_fill would
    store, the packets left untouched (NIC-offload contract; apply on the host
    with tx_apply / tx_apply_batch)."""
    torch = _torch()
    if out is None:
        out = torch.empty(n, dtype=torch.uint32, device=arena.device)
    if flags is None:
        flags = torch.empty(n, dtype=torch.uint8, device=arena.device)
    rc = _lib.lib().tcsum_batch_ipv4_tx_offload(arena.data_ptr(), pkts.data_ptr(), n, out.data_ptr(),
                                                flags.data_ptr(), total_bytes, _stream_ptr(stream))
    _lib.check(rc, "tcsum_batch_ipv4_tx_offload")
    return out, flags


def tx_apply_batch(host_arena: np.ndarray, pkts: np.ndarray, out: np.ndarray, flags: np.ndarray) -> None:
    """Store the offloaded tx values into host frames (tcsum_tx_apply_batch), in place."""
    assert pkts.dtype == PKT_DTYPE
    pkts = np.ascontiguousarray(pkts)
    out = np.ascontiguousarray(out, dtype=np.uint32)
    flags = np.ascontiguousarray(flags, dtype=np.uint8)
    assert out.size == pkts.size and flags.size == pkts.size
    p, nb = _host_arena_args(host_arena)
    _lib.check(_lib.lib().tcsum_tx_apply_batch(p, nb, pkts.ctypes.data, pkts.size, out.ctypes.data,
                                               flags.ctypes.data), "tcsum_tx_apply_batch")


def host_batch_ipv4_rx_verify(host_arena, pkts: np.ndarray, device: int = 0, devices=None):
    """(verdict int8 net_err_t, out, flags) for packets in host memory (with
    `devices`: tcsum_host_batch_ipv4_rx_verify_multi)."""
    assert pkts.dtype == PKT_DTYPE
    pkts = np.ascontiguousarray(pkts)
    verdict = np.zeros(pkts.size, np.int8)
    out = np.zeros(pkts.size, np.uint32)
    flags = np.zeros(pkts.size, np.uint8)
    p, nb = _host_arena_args(host_arena)
    if devices is None:
        rc = _lib.lib().tcsum_host_batch_ipv4_rx_verify(device, p, nb, pkts.ctypes.data, pkts.size,
                                                        verdict.ctypes.data, out.ctypes.data, flags.ctypes.data)
    else:
        dp, nd, _keep = _devices(devices)
        rc = _lib.lib().tcsum_host_batch_ipv4_rx_verify_multi(dp, nd, p, nb, pkts.ctypes.data, pkts.size,
                                                              verdict.ctypes.data, out.ctypes.data,
                                                              flags.ctypes.data)
    _lib.check(rc, "tcsum_host_batch_ipv4_rx_verify")
    return verdict, out, flags


def synth_fill(arena, nbytes: int | None = None, byte_base: int = 0, seed: int = 20240807, stream=None):
    n = arena.numel() if nbytes is None else nbytes
    _lib.check(_lib.bench_lib().tcsum_synth_fill(arena.data_ptr(), n, byte_base, seed, _stream_ptr(stream)),
               "tcsum_synth_fill")


def synth_ipv4(arena, pkts, n: int, seed: int = 20240807, stream=None):
    _lib.check(_lib.bench_lib().tcsum_synth_ipv4(arena.data_ptr(), pkts.data_ptr(), n, seed, _stream_ptr(stream)),
               "tcsum_synth_ipv4")


def probe_read(buf, nbytes: int | None = None, sink=None, stream=None):
    """Plain streaming read of `buf` (the roofline's achievable side)."""
    torch = _torch()
    if sink is None:
        sink = torch.zeros(1, dtype=torch.uint32, device=buf.device)
    n = buf.numel() * buf.element_size() if nbytes is None else nbytes
    _lib.check(_lib.bench_lib().tcsum_probe_read(buf.data_ptr(), n, sink.data_ptr(), _stream_ptr(stream)),
               "tcsum_probe_read")
    return sink


def probe_tile(buf, nbytes: int, lanes: int, loads: int, sink=None, stream=None, dep: bool = False):
    """Plain streaming read of `buf` in the product kernels' tile shape
    (tcsum_probe_tile): the ceiling the checksum kernel is compared with;
    dep=True puts each unit's loads behind one dependent 16-B read."""
    torch = _torch()
    if sink is None:
        sink = torch.zeros(1, dtype=torch.uint32, device=buf.device)
    _lib.check(_lib.bench_lib().tcsum_probe_tile(buf.data_ptr(), nbytes, lanes, loads, 1 if dep else 0,
                                                 sink.data_ptr(), _stream_ptr(stream)), "tcsum_probe_tile")
    return sink


def probe_segments(arena, segs, n: int, total_bytes: int, sink=None, stream=None):
    """tcsum_probe_segments: batch_peso's loads with free arithmetic."""
    torch = _torch()
    if sink is None:
        sink = torch.zeros(1, dtype=torch.uint32, device=arena.device)
    _lib.check(_lib.bench_lib().tcsum_probe_segments(arena.data_ptr(), segs.data_ptr(), n, total_bytes, sink.data_ptr(),
                                               _stream_ptr(stream)), "tcsum_probe_segments")
    return sink


def probe_ipv4(arena, pkts, n: int, total_bytes: int, rx: bool = False, sink=None, stream=None, tx: bool = False,
               masked: bool = False):
    """tcsum_probe_ipv4: the IPv4 batch calls' loads with free arithmetic;
    tx=True adds the deferred tx fill's scratch writes and field scatter (the
    fields are left junk); masked=True: the sums loads with the slots past a
    packet's last chunk masked off instead of clamped."""
    torch = _torch()
    if sink is None:
        sink = torch.zeros(1, dtype=torch.uint32, device=arena.device)
    mode = 3 if masked else 2 if tx else 1 if rx else 0
    _lib.check(_lib.bench_lib().tcsum_probe_ipv4(arena.data_ptr(), pkts.data_ptr(), n, total_bytes, mode,
                                           sink.data_ptr(), _stream_ptr(stream)), "tcsum_probe_ipv4")
    return sink


def txfloor_prepare(arena, nbytes: int, pkts, n: int, total_bytes: int, stream=None) -> dict:
    """tcsum_probe_txfloor_prepare: the tx fill's field addresses and
    16-KiB-window index, for probe_txfloor (outside any measurement)."""
    torch = _torch()
    dev = arena.device
    nw = int(_lib.bench_lib().tcsum_probe_txfloor_windows(nbytes))
    h = dict(arena=arena, nbytes=nbytes, n=n, side=torch.zeros(2 * max(n, 1), dtype=torch.uint32, device=dev),
             fpos=torch.zeros(2 * max(n, 1), dtype=torch.int64, device=dev),
             ffirst=torch.zeros(nw + 1, dtype=torch.uint32, device=dev),
             sink=torch.zeros(1, dtype=torch.uint32, device=dev))
    _lib.check(_lib.bench_lib().tcsum_probe_txfloor_prepare(
        arena.data_ptr(), nbytes, pkts.data_ptr(), n, total_bytes, h["side"].data_ptr(), h["side"].numel(),
        h["fpos"].data_ptr(), h["fpos"].numel(), h["ffirst"].data_ptr(), h["ffirst"].numel(), _stream_ptr(stream)),
        "tcsum_probe_txfloor_prepare")
    return h


def probe_txfloor(h: dict, deferred: bool = False, stream=None, variant: int | None = None):
    """tcsum_probe_txfloor: one read of the batch's bytes plus the fill's
    field writes, in-stream (deferred=False) or as one dense scatter.
    variant 2-7: the read, then a scatter writing each field's aligned block
    of 2 / 16 / 32 / 64 / 128 / 256 bytes (junk around the fields); 8: the
    read, then a read-modify-write of each field's whole 64-B line; 9: the
    fields by device atomics; 10: each field's line loaded, then 2-B stores;
    11: the dword at each field loaded, then 2-B stores; 12 / 13: in-stream,
    each field's 64-B line written whole (junk) / its dword loaded first."""
    v = variant if variant is not None else 1 if deferred else 0
    _lib.check(_lib.bench_lib().tcsum_probe_txfloor(
        h["arena"].data_ptr(), h["nbytes"], h["fpos"].data_ptr(), h["side"].data_ptr(), h["n"],
        h["ffirst"].data_ptr(), v, h["sink"].data_ptr(), _stream_ptr(stream)),
        "tcsum_probe_txfloor")


def pick_geometry(mean_len: int):
    g, u = ctypes.c_int(), ctypes.c_int()
    _lib.lib().tcsum_pick_geometry(mean_len, ctypes.byref(g), ctypes.byref(u))
    return g.value, u.value


def route(mean_len: int) -> dict:
    """The route the batch calls take for a mean range length (debug knobs
    applied): lanes, loads, xcd, packed K (0 = off), and the packed K of a
    SHUFFLED batch (0 = the per-range kernel) (tcsum_debug_route)."""
    r = (ctypes.c_int32 * 5)()
    _lib.lib().tcsum_debug_route(mean_len, r)
    return dict(zip(("lanes", "loads", "xcd", "packed", "shuffled_packed"), list(r)))


def ipv4_route(mean_len: int, ip_mode: int = 0):
    """(lanes, loads) of the k_ipv4 launch an IPv4 batch of this mean packet
    length takes (tcsum_debug_ipv4_route; ip_mode 0 sums, 1 tx fill, 2 rx
    verify, 3 tx offload; debug knobs applied)."""
    r = (ctypes.c_int32 * 2)()
    _lib.lib().tcsum_debug_ipv4_route(mean_len, ip_mode, r)
    return r[0], r[1]


def flat_ipv4(mode: int, arena, pkts, n: int, total_bytes: int, out=None, flags=None, verdict=None, stream=None):
    """The byte-window stream (libtcsum_bench.so's tcsum_flat_ipv4, measurement
    and tests only): mode 0 sums, 1 tx fill, 2 rx verify, 3 tx offload, 4 tx
    fill with deferred stores; device tensors, as the tcsum_batch_ipv4* calls."""
    ptr = lambda t: t.data_ptr() if t is not None else None  # noqa: E731
    rc = _lib.bench_lib().tcsum_flat_ipv4(mode, arena.data_ptr(), pkts.data_ptr(), n, total_bytes, ptr(out),
                                          ptr(flags), ptr(verdict), _stream_ptr(stream))
    _lib.check(rc, "tcsum_flat_ipv4")


def debug_set(key: str, value: int) -> None:
    """Force a route knob for this process (include/tcsum_debug.h; tests and
    measurement only; -1 gives the choice back to the router)."""
    _lib.check(_lib.lib().tcsum_debug_set(key.encode(), int(value)), f"tcsum_debug_set({key})")


def debug_get(key: str) -> int:
    return int(_lib.lib().tcsum_debug_get(key.encode()))


SHARD_DTYPE = np.dtype([("device", "<i4"), ("rc", "<i4"), ("first", "<u4"), ("count", "<u4"), ("bytes", "<u8"),
                        ("ms", "<f8")])


def last_shards() -> list:
    """Per shard of the last multi-device host batch (tcsum_debug_shards):
    device, rc, first, count, bytes, ms."""
    L = _lib.lib()
    k = L.tcsum_debug_shards(None, 0)
    st = np.zeros(max(k, 1), SHARD_DTYPE)
    k = L.tcsum_debug_shards(st.ctypes.data, st.size)
    return [{f: st[f][i].item() for f in SHARD_DTYPE.names} for i in range(k)]


class debug:
    """Context manager: `with tc.debug(lanes=16, loads=6): ...` sets the knobs
    and restores their previous values on exit."""

    def __init__(self, **knobs):
        self.knobs = knobs
        self.saved = {}

    def __enter__(self):
        for k, v in self.knobs.items():
            self.saved[k] = debug_get(k)
            debug_set(k, -1 if v is None else v)
        return self

    def __exit__(self, *exc):
        for k, v in self.saved.items():
            debug_set(k, v)
        return False


def device_count() -> int:
    return _lib.lib().tcsum_device_count()


def release(device: int = 0) -> None:
    """Free the buffers the batch calls cache on `device` (tcsum_release)."""
    _lib.check(_lib.lib().tcsum_release(device), "tcsum_release")


def plat_init(device: int = 0) -> None:
    _lib.check(_lib.lib().tcsum_plat_init(device), "tcsum_plat_init")


def queue_server(enable: bool, device: int = 0) -> None:
    """Serve small host-queue batches from a resident grid (tcsum_queue_server)."""
    _lib.check(_lib.lib().tcsum_queue_server(device, 1 if enable else 0), "tcsum_queue_server")


def call_server(enable: bool, device: int = 0) -> None:
    """Serve the synchronous drop-in calls from one resident wave (tcsum_call_server)."""
    _lib.check(_lib.lib().tcsum_call_server(device, 1 if enable else 0), "tcsum_call_server")
