"""What would configs[1]'s bytes stream at in the TSO kernel's load shape?

One process, one arena (configs[1]: 1M x 1500 B packed, 1.5 GB).  Interleaved
rounds of:
  mtu     tcsum_batch_peso on the 1M x 1500-B descriptors (the headline)
  as64k   tcsum_batch_peso on 24,000 x 64-KiB descriptors covering the SAME
          bytes (k_segments_wgx<16,32,4>: the TSO shape)
  probe   tcsum_probe_segments on the headline descriptors
  read    tcsum_probe_read over the arena
Median us per launch; GB/s priced on the bytes each reads.  The gap between
mtu and as64k is what a packed-stream kernel for 1500-B ranges could win.

  python scripts/mtu_stream_ceiling.py
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


def per_launch(fn, reps=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


b = workload.make_batch("mtu")
arena, descs = workload.materialize(b)
out = torch.empty(b.n, dtype=torch.uint16, device="cuda")
sink = torch.zeros(1, dtype=torch.uint32, device="cuda")
bytes_mtu = b.total_bytes + 26 * b.n


def as_ranges(L):
    n = b.total_bytes // L
    d = np.zeros(n, PESO_DTYPE)
    d["offset"] = np.arange(n, dtype=np.uint64) * np.uint64(L)
    d["len"] = L
    d["protocol"] = 6
    dd = tc.descs_to_device(d)
    o = torch.empty(n, dtype=torch.uint16, device="cuda")
    return (lambda: tc.batch_peso(arena, dd, n, n * L, out=o)), n * (L + 26)


legs = {
    "mtu": (lambda: tc.batch_peso(arena, descs, b.n, b.total_bytes, out=out), bytes_mtu),
    "as64k": as_ranges(65536),
    "as32k": as_ranges(32768),
    "as6000": as_ranges(6000),
    "probe": (lambda: tc.probe_segments(arena, descs, b.n, b.total_bytes, sink=sink), bytes_mtu),
    "read": (lambda: tc.probe_read(arena, b.total_bytes, sink=sink), b.total_bytes),
}
for f, _ in legs.values():
    for _ in range(30):
        f()
torch.cuda.synchronize()
ts = {k: [] for k in legs}
for r in range(9):
    for k, (f, _) in legs.items():
        ts[k].append(per_launch(f))
for k, (f, nb) in legs.items():
    us = float(np.median(ts[k]))
    print(f"{k:6s} {us:9.1f} us  {nb / us / 1e3:8.1f} GB/s  frac {nb / us / 1e3 / 8000:.4f}  "
          f"(min {min(ts[k]):.1f} max {max(ts[k]):.1f})", flush=True)
