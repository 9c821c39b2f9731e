"""Would the packed stream (k_segments_pk) carry configs[3]'s packets faster
than k_ipv4's lane group per packet?  configs[3]'s packet byte ranges as
checksum_peso descriptors (same offsets and lengths, same arena), summed
  ipv4      tcsum_batch_ipv4 (k_ipv4<32,6>: the route, header parse included)
  pk        tcsum_batch_peso, the packed stream (K ranges per workgroup)
  pk=K      the same with K forced
  range     tcsum_batch_peso per range (packed=0: k_segments)
  as64k     the arena as 64-KiB ranges (the TSO shape: the ceiling)
One process, interleaved rounds, the first-timed leg rotated.

  python scripts/ipv4_as_peso.py [config]   (mixed | mixed_aligned)
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tcp_amd as tc  # noqa: E402
from tcp_amd import workload  # noqa: E402
from tcp_amd.csum import PESO_DTYPE  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "mixed"
b = workload.make_batch(cfg)
arena, descs = workload.materialize(b)
d = np.zeros(b.n, PESO_DTYPE)
d["offset"], d["len"], d["protocol"] = b.descs["offset"], b.descs["len"], 6
pd = tc.descs_to_device(d)
o16 = torch.empty(b.n, dtype=torch.uint16, device="cuda")
o32 = torch.empty(b.n, dtype=torch.uint32, device="cuda")
L = 65536
n64 = b.total_bytes // L
d64 = np.zeros(n64, PESO_DTYPE)
d64["offset"], d64["len"], d64["protocol"] = np.arange(n64, dtype=np.uint64) * np.uint64(L), L, 6
dd64 = tc.descs_to_device(d64)
o64 = torch.empty(n64, dtype=torch.uint16, device="cuda")


def knobbed(fn, **kn):
    def g():
        with tc.debug(**kn):
            fn()
    return g


peso = lambda: tc.batch_peso(arena, pd, b.n, b.total_bytes, out=o16)  # noqa: E731
legs = {
    "ipv4": (lambda: tc.batch_ipv4(arena, descs, b.n, b.total_bytes, out=o32, want_flags=False),
             b.total_bytes + 20 * b.n),
    "pk": (peso, b.total_bytes + 26 * b.n),
    "pk=2": (knobbed(peso, packed=2), b.total_bytes + 26 * b.n),
    "pk=4": (knobbed(peso, packed=4), b.total_bytes + 26 * b.n),
    "pk=8": (knobbed(peso, packed=8), b.total_bytes + 26 * b.n),
    "range": (knobbed(peso, packed=0), b.total_bytes + 26 * b.n),
    "as64k": (lambda: tc.batch_peso(arena, dd64, n64, n64 * L, out=o64), n64 * (L + 26)),
}
print("# route for the mean length:", tc.route(b.total_bytes // b.n), flush=True)
for f, _ in legs.values():
    for _ in range(5):
        f()
torch.cuda.synchronize()
names = list(legs)
ts = {k: [] for k in names}
for r in range(7):
    for i in range(len(names)):
        k = names[(r + i) % len(names)]
        f = legs[k][0]
        f()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            f()
        e1.record()
        torch.cuda.synchronize()
        ts[k].append(e0.elapsed_time(e1) / 10 * 1e3)
print(f"# {cfg}: {b.n} packets, {b.total_bytes} B; 7 rounds x 10 launches, first-timed rotated", flush=True)
for k in names:
    us = float(np.median(ts[k]))
    nb = legs[k][1]
    print(f"{k:8s} {us:8.1f} us  {nb / us / 1e3:8.1f} GB/s  frac {nb / us / 1e3 / 8000:.4f}", flush=True)
