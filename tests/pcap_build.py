"""Test helper: write classic libpcap savefiles (the format netif_pcap's
captures are saved in) around given L3 frames, and remember where every
frame's IPv4 header landed -- the expected index, computed independently of
tcsum_pcap_index."""
from __future__ import annotations

import struct

import numpy as np

ETHER, RAW, NULL, SLL, IPV4 = 1, 101, 0, 113, 228
_L2 = {ETHER: 14, RAW: 0, IPV4: 0, NULL: 4, SLL: 16}


def l2_header(link: int, ethertype: int, big_endian: bool) -> bytes:
    if link == ETHER:
        return bytes.fromhex("00163e000001" "00163e000002") + struct.pack(">H", ethertype)
    if link == SLL:
        return struct.pack(">HHH8sH", 0, 1, 6, bytes(8), ethertype)
    if link == NULL:  # AF_INET = 2 for IPv4, 24 (AF_INET6 on BSD) otherwise
        return struct.pack(">I" if big_endian else "<I", 2 if ethertype == 0x0800 else 24)
    return b""


def build(frames, link: int = ETHER, big_endian: bool = False, nanosecond: bool = False,
          ethertypes=None, fcs_len: int = 0, caplen_cut=None):
    """frames: list of L3 payloads (bytes).  Returns (file bytes, expected
    offsets of each IPv4 header in the file, captured L3 lengths)."""
    e = ">" if big_endian else "<"
    magic = 0xA1B23C4D if nanosecond else 0xA1B2C3D4
    linkfield = link | ((1 << 26) | ((fcs_len // 2) << 28) if fcs_len else 0)
    out = bytearray(struct.pack(e + "IHHiIII", magic, 2, 4, 0, 0, 262144, linkfield))
    offs, lens = [], []
    for i, f in enumerate(frames):
        et = 0x0800 if ethertypes is None else ethertypes[i]
        rec = l2_header(link, et, big_endian) + bytes(f) + bytes(range(fcs_len))
        orig = len(rec)
        cap = orig if caplen_cut is None or caplen_cut[i] is None else caplen_cut[i]
        rec = rec[:cap]
        out += struct.pack(e + "IIII", i, 0, cap, orig)
        offs.append(len(out) + _L2[link])
        lens.append(max(0, cap - fcs_len - _L2[link]))
        out += rec
    return bytes(out), np.array(offs, np.uint64), np.array(lens, np.uint32)
