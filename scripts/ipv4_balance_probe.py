"""Is k_ipv4's distance from the TSO shape on configs[3] (0.934 vs ~0.95 of
spec) the length spread inside a workgroup?  A workgroup holds 8 packets (one
per 32-lane group); it lives as long as its longest packet's passes, while
the groups of its short packets idle.  Same byte count in every leg
(~4.75 GB), one process, interleaved rounds, first-timed leg rotated:

  mixed         configs[3]: lengths uniform in [64, 9000], arena order
  sorted        the same lengths sorted: every workgroup's packets alike
  u4532         every packet 4,532 B (configs[3]'s mean)
  u2900         2,900 B: one 3-KiB pass per packet, whatever its line offset
  u5900         5,900 B: two passes
  as64k         the mixed arena as 64-KiB ranges through the TSO kernel
                (checksum_peso over the same bytes; the ceiling)
sums with the route's k_ipv4<32,6> and rx with its k_ipv4<16,6> each.

  python scripts/ipv4_balance_probe.py [ROUNDS]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tcp_amd as tc  # noqa: E402
from tcp_amd import workload  # noqa: E402
from tcp_amd.csum import PESO_DTYPE, PKT_DTYPE  # noqa: E402

TOTAL = workload.make_batch("mixed").total_bytes


def batch_of(lens):
    lens = np.asarray(lens, np.uint64)
    n = lens.size
    offs = np.zeros(n, np.uint64)
    np.cumsum(lens[:-1], out=offs[1:])
    d = np.zeros(n, PKT_DTYPE)
    d["offset"], d["len"] = offs, lens.astype(np.uint32)
    arena = int(offs[-1] + lens[-1])
    return workload.Batch("mixed", "ipv4", n, d, arena, int(lens.sum()), 0)


def per_launch(fn, reps=10):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


mixed = workload.make_batch("mixed")
lens_m = mixed.descs["len"].astype(np.uint64)
batches = {
    "mixed": mixed,
    "sorted": batch_of(np.sort(lens_m)),
    "u4532": batch_of(np.full(TOTAL // 4532, 4532)),
    "u2900": batch_of(np.full(TOTAL // 2900, 2900)),
    "u5900": batch_of(np.full(TOTAL // 5900, 5900)),
}
legs = {}
for name, b in batches.items():
    arena, descs = workload.materialize(b)
    out = torch.empty(b.n, dtype=torch.int32, device="cuda")
    ver = torch.empty(b.n, dtype=torch.int8, device="cuda")
    nb = b.total_bytes + 20 * b.n  # bytes + 16-B descriptor + 4-B result per packet
    legs[f"{name}:sums"] = ((lambda a=arena, d=descs, b=b, o=out: tc.batch_ipv4(a, d, b.n, b.total_bytes, out=o,
                                                                                   want_flags=False)), nb)
    legs[f"{name}:rx"] = ((lambda a=arena, d=descs, b=b, v=ver: tc.batch_ipv4_rx_verify(
        a, d, b.n, b.total_bytes, verdict=v, want_flags=False)), b.total_bytes + 17 * b.n)
    if name == "mixed":
        L = 65536
        n64 = b.total_bytes // L
        d64 = np.zeros(n64, PESO_DTYPE)
        d64["offset"] = np.arange(n64, dtype=np.uint64) * np.uint64(L)
        d64["len"] = L
        d64["protocol"] = 6
        dd = tc.descs_to_device(d64)
        o64 = torch.empty(n64, dtype=torch.uint16, device="cuda")
        legs["mixed:as64k"] = ((lambda a=arena, dd=dd, n64=n64, o=o64: tc.batch_peso(a, dd, n64, n64 * L, out=o)),
                               n64 * (L + 26))
for f, _ in legs.values():
    for _ in range(5):
        f()
torch.cuda.synchronize()
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
names = list(legs)
ts = {k: [] for k in names}
for r in range(rounds):
    for i in range(len(names)):
        k = names[(r + i) % len(names)]
        ts[k].append(per_launch(legs[k][0]))
print(f"# {rounds} rounds x 10 launches, first-timed leg rotated; GB/s of algorithmic bytes", flush=True)
for k in names:
    us = float(np.median(ts[k]))
    nb = legs[k][1]
    print(f"{k:14s} {us:8.1f} us  {nb / us / 1e3:8.1f} GB/s  frac {nb / us / 1e3 / 8000:.4f}", flush=True)
