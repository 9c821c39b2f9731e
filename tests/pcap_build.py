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


def _pad4(b: bytes) -> bytes:
    return b + bytes(-len(b) % 4)


def build_ng(frames, links=(ETHER,), iface_of=None, big_endian: bool = False, block="epb", fcs_bits=None,
             extra_blocks: bool = True, sections=1):
    """A pcapng file: `sections` Section Header Blocks, each followed by one
    Interface Description Block per entry of `links` and the frames (split
    evenly over the sections) as Enhanced ("epb"), Simple ("spb") or obsolete
    ("pb") Packet Blocks; with extra_blocks, a Name Resolution Block and an
    Interface Statistics Block are mixed in.  Returns (file bytes, expected
    IPv4 offsets, captured L3 lengths)."""
    e = ">" if big_endian else "<"

    def blk(btype: int, body: bytes) -> bytes:
        body = _pad4(body)
        n = 12 + len(body)
        return struct.pack(e + "II", btype, n) + body + struct.pack(e + "I", n)

    out = bytearray()
    offs, lens = [], []
    per = -(-len(frames) // max(1, sections))
    for s_ in range(sections):
        out += blk(0x0A0D0D0A, struct.pack(e + "IHHq", 0x1A2B3C4D, 1, 0, -1))
        for link in links:
            opts = b""
            if fcs_bits is not None:
                opts = struct.pack(e + "HH", 13, 1) + bytes([fcs_bits]) + bytes(3) + struct.pack(e + "HH", 0, 0)
            out += blk(1, struct.pack(e + "HHI", link, 0, 262144) + opts)
        if extra_blocks:
            out += blk(4, struct.pack(e + "HH", 0, 0))  # empty NRB
        fcs = (fcs_bits or 0) // 8
        for i in range(s_ * per, min(len(frames), (s_ + 1) * per)):
            itf = 0 if iface_of is None else iface_of[i]
            link = links[itf]
            rec = l2_header(link, 0x0800, big_endian) + bytes(frames[i]) + bytes(range(fcs))
            if block == "epb":
                hdr = struct.pack(e + "IIIII", itf, 0, i, len(rec), len(rec))
                data_at = len(out) + 8 + 20
                out += blk(6, hdr + rec)
            elif block == "pb":
                hdr = struct.pack(e + "HHIIII", itf, 0, 0, i, len(rec), len(rec))
                data_at = len(out) + 8 + 20
                out += blk(2, hdr + rec)
            else:
                data_at = len(out) + 8 + 4
                out += blk(3, struct.pack(e + "I", len(rec)) + rec)
            offs.append(data_at + _L2.get(link, 0))
            lens.append(len(rec) - fcs - _L2.get(link, 0))
            if extra_blocks and i % 97 == 5:
                out += blk(5, struct.pack(e + "III", itf, 0, 0))  # ISB
    return bytes(out), np.array(offs, np.uint64), np.array(lens, np.uint32)
