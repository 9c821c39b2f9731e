"""Per-launch time of 200 back-to-back configs[1] launches, the headline
kernel vs the plain read probe on the same bytes (measurement script): does
the kernel slow down under sustained load, and does the probe?"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tcp_amd as tc  # noqa: E402
from tcp_amd import workload  # noqa: E402

b = workload.make_batch("mtu")
arena, descs = workload.materialize(b)
out = torch.empty(b.n, dtype=torch.uint16, device="cuda")
sink = torch.zeros(1, dtype=torch.uint32, device="cuda")
K = 200
for name, f in (("kernel", lambda: tc.batch_peso(arena, descs, b.n, b.total_bytes, out=out)),
                ("probe", lambda: tc.probe_read(arena, b.arena_bytes, sink)),
                ("kernel again", lambda: tc.batch_peso(arena, descs, b.n, b.total_bytes, out=out))):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(K + 1)]
    ev[0].record()
    for i in range(K):
        f()
        ev[i + 1].record()
    torch.cuda.synchronize()
    t = np.array([ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(K)])
    print(f"{name:13s} mean {t.mean():6.1f} us; by 20-launch block: "
          + " ".join(f"{t[i:i + 20].mean():5.1f}" for i in range(0, K, 20)), flush=True)
