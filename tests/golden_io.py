"""Readers for the golden fixtures in tests/golden/.

The fixtures were produced by the reference compiled from /root/reference by
``make -C oracle golden``:

* oracle/golden_gen.c -- the reference's own checksum16 / pktbuf_checksum16 /
  checksum_peso (net/src/tools.c:24-75, net/src/pktbuf.c:646-670) on recorded
  inputs (flat, pktbuf, peso, ipv4 sums, ipv4_tx on malformed packets);
* oracle/stack_gen.c -- the whole reference stack: frames its transmit path
  built and checksummed (stack_tx_*), and the net_err_t its receive path
  returns for each rx frame (ipv4_rx_*).

They are plain little-endian u32 records; the layouts below mirror the
generators.
"""
from __future__ import annotations

import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

FLAT = np.dtype([("pool_off", "<u4"), ("len", "<u4"), ("offset", "<i4"), ("pre_sum", "<u4"),
                 ("complement", "<u4"), ("expected", "<u4")])
PKTBUF = np.dtype([("pool_off", "<u4"), ("total", "<u4"), ("blk_first", "<u4"), ("nblk", "<u4"),
                   ("seek", "<u4"), ("len", "<i4"), ("pre_sum", "<i4"), ("complement", "<u4"),
                   ("expected", "<u4"), ("final_pos", "<u4"), ("final_blk", "<u4"),
                   ("final_blk_off", "<u4")])
PESO = np.dtype([("pool_off", "<u4"), ("total", "<u4"), ("blk_first", "<u4"), ("nblk", "<u4"),
                 ("src", "u1", 4), ("dst", "u1", 4), ("proto", "<u4"), ("expected", "<u4"),
                 ("final_pos", "<u4"), ("final_blk", "<u4")])
IPV4 = np.dtype([("pool_off", "<u4"), ("frame_len", "<u4"), ("ip", "<u4"), ("l4", "<u4"),
                 ("flags", "<u4")])

IPV4_TX = np.dtype([("pool_off", "<u4"), ("frame_len", "<u4"), ("flags", "<u4")])
# gate & 0xFF: which reference function decided (1 ipv4_in's own checks,
# 2 fragment queued for reassembly, 3 the L4 input tcp_in/udp_in/icmpv4_in/
# raw_in); gate >> 8: the packet's protocol byte
IPV4_RX = np.dtype([("pool_off", "<u4"), ("frame_len", "<u4"), ("verdict", "<i4"), ("flags", "<u4"),
                    ("gate", "<u4")])
# kind >> 8: protocol; kind & 1: a fragment (only its header checksum is filled)
STACK_TX = np.dtype([("pool_off", "<u4"), ("frame_len", "<u4"), ("flags", "<u4"), ("kind", "<u4")])

NO_BLOCK = 0xFFFFFFFF


def _load(name: str, dtype=np.uint8) -> np.ndarray:
    return np.fromfile(os.path.join(GOLDEN, name), dtype=dtype)


def pool() -> np.ndarray:
    return _load("pool.bin")


def flat_cases() -> np.ndarray:
    return _load("flat_cases.bin", FLAT)


def pktbuf_cases():
    return _load("pktbuf_cases.bin", PKTBUF), _load("pktbuf_blocks.bin", np.uint32)


def peso_cases():
    return _load("peso_cases.bin", PESO), _load("peso_blocks.bin", np.uint32)


def ipv4_cases():
    return _load("ipv4_cases.bin", IPV4), _load("ipv4_pool.bin")


def ipv4_tx_cases():
    """(cases, pool before the fill, pool after the reference's fill)."""
    return _load("ipv4_tx_cases.bin", IPV4_TX), _load("ipv4_tx_in.bin"), _load("ipv4_tx_out.bin")


def stack_tx_cases():
    """Frames the reference stack transmitted: (cases, frames with the filled
    checksum fields junked, frames as the reference sent them)."""
    return _load("stack_tx_cases.bin", STACK_TX), _load("stack_tx_in.bin"), _load("stack_tx_out.bin")


def ipv4_rx_cases():
    return _load("ipv4_rx_cases.bin", IPV4_RX), _load("ipv4_rx_pool.bin")


def pkt_descs(cases, dtype):
    d = np.zeros(cases.size, dtype)
    d["offset"] = cases["pool_off"]
    d["len"] = cases["frame_len"]
    return d


def kats() -> dict:
    with open(os.path.join(GOLDEN, "kat.json")) as f:
        return json.load(f)


def kat_inputs() -> dict:
    """The KAT inputs as bytes."""
    k = kats()
    pattern = bytes((i * 7 + 3) & 0xFF for i in range(999))
    return {
        "KAT-1": (bytes.fromhex(k["KAT-1"]["hex"]), k["KAT-1"]["expected"]),
        "KAT-2": (pattern, k["KAT-2"]["expected"]),
        "KAT-3": (pattern, k["KAT-3"]["expected"]),
        "KAT-4": (bytes.fromhex(k["KAT-4"]["hex"]), k["KAT-4"]["expected"]),
        "KAT-5": (bytes.fromhex(k["KAT-5"]["hex"]), k["KAT-5"]["expected"]),
    }


def case_blocks(case, blocks: np.ndarray, data: np.ndarray):
    """Split a case's bytes into the reference's block sizes (chain order)."""
    sizes = blocks[case["blk_first"]: case["blk_first"] + case["nblk"]]
    base = int(case["pool_off"])
    out, at = [], base
    for s in sizes:
        out.append(data[at: at + int(s)])
        at += int(s)
    assert at - base == int(case["total"])
    return out
