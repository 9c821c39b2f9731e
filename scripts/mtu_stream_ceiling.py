"""What would configs[1]'s bytes stream at in the TSO kernel's load shape?

One process.  Interleaved rounds (the leg timed first rotated each round) of:
  mtu       tcsum_batch_peso on the 1M x 1500 B descriptors (the headline):
            reads the 1.573 GB of segments AND the 25.2 MB descriptor array,
            writes 2.1 MB of sums -- 1.6001 GB algorithmic
  as64k     tcsum_batch_peso on 24,000 x 64-KiB descriptors covering the same
            1.573 GB of segment bytes (k_segments_wgx<16,32,4>: the TSO shape);
            its descriptor array is 576 KB
  as64k_eq  the same shape over a buffer as large as everything the headline
            moves (segments + descriptors + sums, 1.6001 GB): the TSO shape
            at the headline's byte count
  read      tcsum_probe_read over the 1.573 GB of segments
  read_eq   tcsum_probe_read over 1.6001 GB
Median us per launch; GB/s priced on the bytes each leg moves.  Round 4's
verdict read the gap between mtu and as64k in microseconds; in bytes per
second it is the descriptor array (profiles/r05/README.md).

  python scripts/mtu_stream_ceiling.py [ROUNDS]
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
bytes_mtu = b.total_bytes + 26 * b.n  # segments + 24-B descriptors + 2-B sums
L = 65536
n_eq = -(-bytes_mtu // (L + 26))  # 64-KiB ranges whose bytes + descriptors + sums match the headline's
big = torch.empty(n_eq * L + 64, dtype=torch.uint8, device="cuda")
big[: arena.numel()].copy_(arena[: min(arena.numel(), big.numel())])


def as_ranges(buf, n):
    d = np.zeros(n, PESO_DTYPE)
    d["offset"] = np.arange(n, dtype=np.uint64) * np.uint64(L)
    d["len"] = L
    d["protocol"] = 6
    dd = tc.descs_to_device(d)
    o = torch.empty(n, dtype=torch.uint16, device="cuda")
    return (lambda: tc.batch_peso(buf, dd, n, n * L, out=o)), n * (L + 26)


legs = {
    "mtu": (lambda: tc.batch_peso(arena, descs, b.n, b.total_bytes, out=out), bytes_mtu),
    "as64k": as_ranges(arena, b.total_bytes // L),
    "as64k_eq": as_ranges(big, n_eq),
    "read": (lambda: tc.probe_read(arena, b.total_bytes, sink=sink), b.total_bytes),
    "read_eq": (lambda: tc.probe_read(big, bytes_mtu // 16 * 16, sink=sink), bytes_mtu // 16 * 16),
}
for f, _ in legs.values():
    for _ in range(30):
        f()
torch.cuda.synchronize()
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 9
names = list(legs)
ts = {k: [] for k in legs}
for r in range(rounds):
    for i in range(len(names)):
        k = names[(r + i) % len(names)]
        ts[k].append(per_launch(legs[k][0]))
print(f"# {rounds} rounds x 20 launches, first-timed leg rotated; bytes moved per launch in brackets", flush=True)
for k, (f, nb) in legs.items():
    us = float(np.median(ts[k]))
    print(f"{k:9s} [{nb / 1e9:.4f} GB] {us:8.1f} us  {nb / us / 1e3:8.1f} GB/s  frac {nb / us / 1e3 / 8000:.4f}  "
          f"(min {min(ts[k]):.1f} max {max(ts[k]):.1f})", flush=True)
