"""k_ipv4's load pattern with the data pass's spare load slots (past a
packet's last chunk) clamped to that chunk, as the route issues them, or
masked off (tcsum_probe_ipv4 modes 0 / 3), beside the product's sums call,
on configs[3] and on equal-length packets.  Interleaved rounds, median.
Measurement script.

  python scripts/ipv4_mask_probe.py [config ...]   (mixed, uNNNN)
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tcp_amd as tc  # noqa: E402
from tcp_amd import workload  # noqa: E402
from tcp_amd.csum import PKT_DTYPE  # noqa: E402


def equal_length(L):
    total = workload.make_batch("mixed").total_bytes
    n = total // L
    d = np.zeros(n, PKT_DTYPE)
    d["offset"] = np.arange(n, dtype=np.uint64) * np.uint64(L)
    d["len"] = L
    return workload.Batch("mixed", "ipv4", n, d, n * L, n * L, 0, op="sums")


s = torch.cuda.current_stream()
for cfg in sys.argv[1:] or ["mixed", "u300", "u1000", "u2900"]:
    b = equal_length(int(cfg[1:])) if cfg.startswith("u") else workload.make_batch(cfg)
    arena, descs = workload.materialize(b)
    out = torch.empty(b.n, dtype=torch.uint32, device="cuda")
    sink = torch.zeros(1, dtype=torch.uint32, device="cuda")
    legs = {"product sums": lambda: tc.batch_ipv4(arena, descs, b.n, b.total_bytes, out=out, want_flags=False),
            "loads, spare slots clamped": lambda: tc.probe_ipv4(arena, descs, b.n, b.total_bytes, sink=sink),
            "loads, spare slots masked": lambda: tc.probe_ipv4(arena, descs, b.n, b.total_bytes, sink=sink,
                                                                masked=True)}
    names = list(legs)
    ts = {k: [] for k in names}
    for r in range(7):
        for i in range(len(names)):
            k = names[(r + i) % len(names)]
            legs[k]()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(10):
                legs[k]()
            e1.record(s)
            torch.cuda.synchronize()
            ts[k].append(e0.elapsed_time(e1) / 10 * 1e3)
    print(f"# {cfg}: {b.n} packets, {b.total_bytes} B; median of 7 interleaved rounds x 10", flush=True)
    for k in names:
        v = float(np.median(ts[k]))
        print(f"  {k:28s} {v:8.1f} us  {b.total_bytes / (v * 1e-6) / 8e12:.4f} of 8 TB/s", flush=True)
    del arena, descs
    torch.cuda.empty_cache()
