"""The tx fill's two forms (debug tx_split 0 = stores in k_ipv4, 1 = deferred
to k_tx_scatter) and the offload form on equal-length IPv4 packets of
configs[3]'s bytes: which form short packets want.  Interleaved rounds,
median.  Measurement script.

  python scripts/tx_short_probe.py [LEN ...]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tcp_amd as tc  # noqa: E402
from tcp_amd import workload  # noqa: E402
from tcp_amd.csum import PKT_DTYPE  # noqa: E402

s = torch.cuda.current_stream()
for L in [int(a) for a in sys.argv[1:]] or [100, 300, 1000, 3000]:
    total = workload.make_batch("mixed").total_bytes
    n = total // L
    d = np.zeros(n, PKT_DTYPE)
    d["offset"] = np.arange(n, dtype=np.uint64) * np.uint64(L)
    d["len"] = L
    b = workload.Batch("mixed", "ipv4", n, d, n * L, n * L, 0, op="sums")
    arena, descs = workload.materialize(b)
    out = torch.empty(n, dtype=torch.uint32, device="cuda")
    fl = torch.empty(n, dtype=torch.uint8, device="cuda")

    def fill(split):
        with tc.debug(tx_split=split):
            tc.batch_ipv4_tx_fill(arena, descs, n, b.total_bytes, want_flags=False)

    legs = {"fill, stores in the kernel": lambda: fill(0), "fill, deferred stores": lambda: fill(1),
            "offload (no stores)": lambda: tc.batch_ipv4_tx_offload(arena, descs, n, b.total_bytes, out=out, flags=fl),
            "sums": lambda: tc.batch_ipv4(arena, descs, n, b.total_bytes, out=out, want_flags=False)}
    names = list(legs)
    ts = {k: [] for k in names}
    for r in range(5):
        for i in range(len(names)):
            k = names[(r + i) % len(names)]
            legs[k]()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(5):
                legs[k]()
            e1.record(s)
            torch.cuda.synchronize()
            ts[k].append(e0.elapsed_time(e1) / 5 * 1e3)
    print(f"# {L}-B packets: {n}, median of 5 interleaved rounds x 5", flush=True)
    for k in names:
        v = float(np.median(ts[k]))
        print(f"  {k:28s} {v:9.1f} us  {b.total_bytes / (v * 1e-6) / 8e12:.4f} of 8 TB/s", flush=True)
    del arena, descs
    torch.cuda.empty_cache()
