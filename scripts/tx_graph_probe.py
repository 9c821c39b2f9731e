"""tx fill on configs[3] captured in a hipGraph: the single-launch form the
plain call takes under capture, against the deferred-store form with caller
scratch (tcsum_batch_ipv4_tx_fill_scratch).  Interleaved rounds of graph
replays, median us per fill.  Measurement script, not product code."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tcp_amd as tc  # noqa: E402
from tcp_amd import workload  # noqa: E402

b = workload.make_batch("mixed_tx")
arena, descs = workload.materialize(b)
scratch = torch.empty(8 * b.n, dtype=torch.uint8, device="cuda")
K = 10
graphs = {}
s = torch.cuda.Stream()
for name, kw in (("single launch (capture)", {}), ("deferred, caller scratch", {"scratch": scratch})):
    tc.batch_ipv4_tx_fill(arena, descs, b.n, b.total_bytes, want_flags=False, **kw)  # warm
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(K):
            tc.batch_ipv4_tx_fill(arena, descs, b.n, b.total_bytes, want_flags=False, **kw)
    graphs[name] = g
per = {k: [] for k in graphs}
for r in range(7):
    for name, g in (graphs.items() if r % 2 == 0 else reversed(list(graphs.items()))):
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        per[name].append(e0.elapsed_time(e1) * 1e3 / K)
print(f"# mixed_tx: {b.n} packets, {b.total_bytes} B; {K} fills per graph, median of 7 interleaved rounds")
base = None
for name, v in per.items():
    m = float(np.median(v))
    base = base or m
    print(f"{name:28s} {m:8.1f} us  {m / base:.3f}x")
