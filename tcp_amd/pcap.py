"""Capture files on the rx path: a libpcap savefile's bytes are the arena.

`index` wraps tcsum_pcap_index (include/tcsum_pcap.h, libtcsum_pcap.so): one descriptor per record,
pointing at the record's IPv4 packet inside the file, plus what the stack's
rx front end does with the frame before ipv4_in (plat/netif_pcap.c:9-38,
net/src/ether.c:14-25,62-101).  `rx_verify` then runs the batched rx gates
(tcsum_host_batch_ipv4_rx_verify, the GPU path) over the file in place and
merges the two verdicts per frame; `tx_fill` fills a capture's checksums in
place by the stack's tx rules.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .csum import PKT_DTYPE, host_batch_ipv4_rx_verify, host_batch_ipv4_tx_fill


def _as_u8(buf) -> np.ndarray:
    a = np.frombuffer(buf, dtype=np.uint8) if not isinstance(buf, np.ndarray) else buf
    assert a.dtype == np.uint8 and a.ndim == 1 and a.flags.c_contiguous
    return a


def index(buf):
    """(pkts PKT_DTYPE[frames], l2_verdict int8[frames]) for a savefile in
    memory (bytes, mmap, or a u8 numpy array); raises on a file that is not
    one, or that ends inside a record."""
    a = _as_u8(buf)
    L = _lib.pcap_lib()
    n = ctypes.c_uint32(0)
    rc = L.tcsum_pcap_index(a.ctypes.data, a.nbytes, None, None, 0, ctypes.byref(n))
    if rc not in (_lib.OK, _lib.ERR_MEM):
        _lib.check(rc, "tcsum_pcap_index")
    pkts = np.zeros(n.value, PKT_DTYPE)
    l2 = np.zeros(n.value, np.int8)
    got = ctypes.c_uint32(0)
    _lib.check(L.tcsum_pcap_index(a.ctypes.data, a.nbytes, pkts.ctypes.data, l2.ctypes.data, n.value,
                                  ctypes.byref(got)), "tcsum_pcap_index")
    assert got.value == n.value
    return pkts, l2


def rx_verify(buf, device: int = 0, devices=None):
    """Per frame of the capture: (verdict int8, l2 int8, out u32, flags u8).
    verdict is the rx front end's (l2) where the frame does not reach
    ipv4_in, else the rx gates' net_err_t (tcsum_batch_ipv4_rx_verify).
    `devices`: shard the frames by bytes over those GPUs."""
    a = _as_u8(buf)
    pkts, l2 = index(a)
    verdict, out, flags = host_batch_ipv4_rx_verify(a, pkts, device, devices)
    verdict = np.where(l2 == _lib.OK, verdict, l2).astype(np.int8)
    return verdict, l2, out, flags


def tx_fill(buf, device: int = 0, devices=None):
    """Fill the IPv4 header and L4 checksums of every frame of a capture that
    reaches ipv4_in, in place, by the stack's tx rules (ipv4.c:643,656,
    tcp_out.c:19-20, udp.c:320-321, icmpv4.c:45-58): a capture's checksums
    fixed the way the stack would have sent them.  Frames the front end does
    not hand to ipv4_in are left alone.  Returns (l2 int8, flags u8)."""
    a = _as_u8(buf)
    assert a.flags.writeable, "tx_fill writes the capture in place"
    pkts, l2 = index(a)
    flags = host_batch_ipv4_tx_fill(a, pkts, device, devices)
    return l2, flags


def _main(argv=None) -> int:
    """python -m tcp_amd.pcap FILE [--fill OUT] [--devices 0,1,...]: verify
    every frame of a capture with the stack's rx rules on the GPU and print
    one count per verdict; with --fill, also write a copy whose checksums are
    filled by the stack's tx rules."""
    import argparse
    import collections

    from . import csum
    names = {0: "OK", -5: "SIZE", -11: "NOT_SUPPORT", -13: "BROKEN", _lib.PCAP_ARP: "ARP (not ipv4_in)"}
    ap = argparse.ArgumentParser(prog="python -m tcp_amd.pcap")
    ap.add_argument("file")
    ap.add_argument("--fill", metavar="OUT")
    ap.add_argument("--devices", default="0")
    args = ap.parse_args(argv)
    devices = [int(x) for x in args.devices.split(",")]
    with open(args.file, "rb") as fh:
        size = fh.seek(0, 2)
        fh.seek(0)
        arena = csum.HostArena(size)  # pinned: read in place by the GPU
        fh.readinto(memoryview(arena.array))
    try:
        verdict, l2, _, _ = rx_verify(arena.array, devices[0], devices if len(devices) > 1 else None)
        counts = collections.Counter(verdict.tolist())
        print(f"{verdict.size} frames: " + ", ".join(f"{names.get(k, k)} {v}" for k, v in sorted(counts.items())))
        if args.fill:
            tx_fill(arena.array, devices[0], devices if len(devices) > 1 else None)
            with open(args.fill, "wb") as out:
                out.write(memoryview(arena.array))
    finally:
        arena.free()
    return 0


if __name__ == "__main__":
    raise SystemExit(_main())
