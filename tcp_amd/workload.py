"""Synthetic packet batches for BASELINE.json's configs, and their per-GPU split.

    mtu    configs[1]  1,048,576 x 1500 B TCP segments            (checksum_peso)
    tso    configs[2]    262,144 x 65,536 B TCP segments          (checksum_peso;
                       the pseudo-header length word is (uint16_t)65536 = 0,
                       exactly as tools.c:69 truncates it)
    mixed  configs[3]  1,048,576 IPv4 packets, total length uniform in
                       [64, 9000] B, TCP/UDP 50/50, packed back to back at
                       unaligned offsets ("aligned" variant: 16-byte starts)
    configs[4] = mtu on every GPU (1M per GPU, 8M over 8 GPUs).

Bytes come from the splitmix64 stream shared with the CPU oracle
(tcsum_synth_fill / orc_synth_fill), generated on the device; descriptors are
built here with numpy.  A rank's packets carry global indices rank*n + i, so
N GPUs together hold one N-times-larger batch (weak scaling, no exchange).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .csum import PESO_DTYPE, PKT_DTYPE

SEED = 20240807
CONFIGS = {
    "mtu": dict(n=1 << 20, len=1500, kind="peso"),
    "tso": dict(n=1 << 18, len=65536, kind="peso"),
    "mixed": dict(n=1 << 20, lo=64, hi=9000, kind="ipv4", aligned=False),
    "mixed_aligned": dict(n=1 << 20, lo=64, hi=9000, kind="ipv4", aligned=True),
    # the same packets through the tx fill / rx verify entry points
    "mixed_tx": dict(n=1 << 20, lo=64, hi=9000, kind="ipv4", aligned=False, op="tx"),
    "mixed_rx": dict(n=1 << 20, lo=64, hi=9000, kind="ipv4", aligned=False, op="rx"),
    "mixed_txo": dict(n=1 << 20, lo=64, hi=9000, kind="ipv4", aligned=False, op="txo"),
}
CONFIG_NAMES = {
    "mtu": "1M x 1500 B TCP segments (MTU), device-resident",
    "tso": "256K x 64 KiB TCP segments (TSO-size), device-resident",
    "mixed": "1M mixed IPv4 TCP/UDP packets, uniform 64-9000 B, packed (unaligned)",
    "mixed_aligned": "1M mixed IPv4 TCP/UDP packets, uniform 64-9000 B, 16-B aligned starts",
    "mixed_tx": "1M mixed IPv4 packets: batched tx fill (checksums written in place)",
    "mixed_rx": "1M mixed IPv4 packets: batched rx verify (net_err_t verdict per packet)",
    "mixed_txo": "1M mixed IPv4 packets: batched tx offload (the fill's values + flags out, packets untouched)",
}


def splitmix64(x: np.ndarray) -> np.ndarray:
    """Vectorised splitmix64 (same constants as the device and oracle)."""
    with np.errstate(over="ignore"):
        z = (x.astype(np.uint64) + np.uint64(0x9E3779B97F4A7C15))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


@dataclass
class Batch:
    config: str
    kind: str            # "peso" or "ipv4"
    n: int
    descs: np.ndarray    # PESO_DTYPE or PKT_DTYPE
    arena_bytes: int     # bytes the packets span (arena is allocated 16-B padded)
    total_bytes: int     # sum of packet lengths (the metric's byte count)
    byte_base: int       # where this rank's arena starts in the global stream
    seed: int = SEED
    op: str = "sums"     # ipv4 only: "sums", "tx" (fill in place) or "rx" (verify)

    @property
    def alloc_bytes(self) -> int:
        return ((self.arena_bytes + 15) // 16) * 16 + 64


def make_batch(config: str, rank: int = 0, n: int | None = None, seed: int = SEED) -> Batch:
    """Descriptors for `config` as held by `rank` (n overrides the count)."""
    spec = CONFIGS[config]
    n = spec["n"] if n is None else n
    gidx = np.arange(n, dtype=np.uint64) + np.uint64(rank * n)
    if spec["kind"] == "peso":
        L = spec["len"]
        d = np.zeros(n, PESO_DTYPE)
        d["offset"] = np.arange(n, dtype=np.uint64) * np.uint64(L)
        d["len"] = L
        h = splitmix64(gidx ^ np.uint64(seed + 1))
        d["src"] = (h & np.uint64(0xFFFFFFFF)).astype("<u4").view(np.uint8).reshape(n, 4)
        d["dst"] = (h >> np.uint64(32)).astype("<u4").view(np.uint8).reshape(n, 4)
        d["protocol"] = 6
        arena = n * L
        total = n * L
    else:
        lo, hi = spec["lo"], spec["hi"]
        lens = (splitmix64(gidx ^ np.uint64(seed + 2)) % np.uint64(hi - lo + 1) + np.uint64(lo)).astype(np.uint64)
        stride = ((lens + np.uint64(15)) // np.uint64(16)) * np.uint64(16) if spec["aligned"] else lens
        offs = np.zeros(n, np.uint64)
        np.cumsum(stride[:-1], out=offs[1:])
        d = np.zeros(n, PKT_DTYPE)
        d["offset"] = offs
        d["len"] = lens.astype(np.uint32)
        arena = int(offs[-1] + stride[-1]) if n else 0
        total = int(lens.sum())
    byte_base = rank * (((arena + 15) // 16) * 16)
    return Batch(config, spec["kind"], n, d, arena, total, byte_base, seed, spec.get("op", "sums"))


def materialize(batch: Batch, device="cuda", stream=None):
    """(arena, descs) on the device: bytes generated in HBM, descriptors copied."""
    import torch

    from .csum import batch_ipv4_tx_fill, descs_to_device, synth_fill, synth_ipv4
    arena = torch.empty(batch.alloc_bytes, dtype=torch.uint8, device=device)
    synth_fill(arena, batch.alloc_bytes, batch.byte_base, batch.seed, stream=stream)
    descs = descs_to_device(batch.descs, device)
    if batch.kind == "ipv4":
        synth_ipv4(arena, descs, batch.n, batch.seed, stream=stream)
        if batch.op == "rx":  # receive what a sender filled in
            batch_ipv4_tx_fill(arena, descs, batch.n, batch.total_bytes, want_flags=False, stream=stream)
    return arena, descs


def shard_bounds(lengths: np.ndarray, world: int) -> np.ndarray:
    """Split packets [0, n) into `world` contiguous ranges of ~equal bytes.

    Returns world+1 packet indices; rank r owns [b[r], b[r+1]).  Used to split
    one global batch for strong scaling (balance by bytes, not
    by count -- it matters for the mixed config).
    """
    n = int(lengths.size)
    if world <= 1 or n == 0:
        return np.array([0, n], dtype=np.int64)
    csum = np.cumsum(lengths.astype(np.uint64))
    total = int(csum[-1])
    targets = [(total * r) // world for r in range(1, world)]
    cuts = np.searchsorted(csum, np.array(targets, dtype=np.uint64), side="right")
    return np.concatenate([[0], cuts.astype(np.int64), [n]])


def rebase(descs: np.ndarray, lo: int, hi: int):
    """The descriptors of packets [lo, hi) with offsets relative to their first
    byte, and the byte range [start, end) of the global arena they need."""
    part = descs[lo:hi].copy()
    if part.size == 0:
        return part, 0, 0
    start = int(part["offset"].min())
    end = int((part["offset"] + part["len"]).max())
    part["offset"] -= np.uint64(start)
    return part, start, end
