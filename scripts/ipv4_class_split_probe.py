"""How much configs[3] (1M IPv4 packets of 64-9000 B) would gain if its
packets were split by length into classes, each launched with the shape the
router gives that class's mean (ipv4_short_shape): the descriptors are
partitioned on the host here, outside the timing, so this is the upper
bound of a device-side partition.  Interleaved rounds, median; the split
launches' results are checked against the single launch's.  Measurement
script.

  python scripts/ipv4_class_split_probe.py [EDGE ...]   (class edges in bytes)
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tcp_amd as tc  # noqa: E402
from tcp_amd import workload  # noqa: E402

edges = [int(a) for a in sys.argv[1:]] or [1300, 2800]
s = torch.cuda.current_stream()
for cfg in ("mixed", "mixed_rx"):
    b = workload.make_batch(cfg)
    arena, descs = workload.materialize(b)
    rx = b.op == "rx"
    lens = b.descs["len"].astype(np.int64)
    cls = np.digitize(lens, edges)
    parts = []
    for c in range(len(edges) + 1):
        idx = np.nonzero(cls == c)[0]
        d = tc.descs_to_device(np.ascontiguousarray(b.descs[idx]))
        parts.append((idx, d, int(idx.size), int(lens[idx].sum())))
    out = torch.empty(b.n, dtype=torch.int8 if rx else torch.uint32, device="cuda")
    outs = [torch.empty(p[2], dtype=torch.int8 if rx else torch.uint32, device="cuda") for p in parts]

    def one(o, d, n, total):
        if rx:
            tc.batch_ipv4_rx_verify(arena, d, n, total, verdict=o, want_flags=False)
        else:
            tc.batch_ipv4(arena, d, n, total, out=o, want_flags=False)

    legs = {"one launch (route)": lambda: one(out, descs, b.n, b.total_bytes),
            f"{len(parts)} class launches": lambda: [one(o, p[1], p[2], p[3]) for o, p in zip(outs, parts)]}
    names = list(legs)
    for k in names:
        legs[k]()
    torch.cuda.synchronize()
    full = out.cpu().numpy()
    for o, p in zip(outs, parts):
        assert np.array_equal(o.cpu().numpy(), full[p[0]])
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
    shapes = [tc.ipv4_route(p[3] // max(p[2], 1), 2 if rx else 0) for p in parts]
    print(f"# {cfg}: edges {edges}, classes {[p[2] for p in parts]} packets, shapes {shapes}; results equal",
          flush=True)
    for k in names:
        v = float(np.median(ts[k]))
        print(f"  {k:24s} {v:8.1f} us  {b.total_bytes / (v * 1e-6) / 8e12:.4f} of 8 TB/s", flush=True)
    del arena, descs
    torch.cuda.empty_cache()
