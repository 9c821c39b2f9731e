"""tcsum_host_batch_peso on configs[1] from a pinned arena (tcsum_host_alloc)
and from a pageable numpy array, same bytes, one process.  Measurement
script, not product code."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tcp_amd as tc  # noqa: E402
from tcp_amd import workload  # noqa: E402

GIB = 1 << 30
b = workload.make_batch("mtu")
arena, descs = workload.materialize(b)
want = tc.batch_peso(arena, descs, b.n, b.total_bytes).cpu().numpy()
ha = tc.HostArena(b.alloc_bytes)
ha.array[:] = arena[: b.alloc_bytes].cpu().numpy()
page = np.array(ha.array)
del arena, descs
torch.cuda.empty_cache()
for name, host in (("pinned", ha.array), ("pageable", page), ("pinned", ha.array), ("pageable", page)):
    out = tc.host_batch_peso(host, b.descs)
    t0 = time.perf_counter()
    for _ in range(3):
        out = tc.host_batch_peso(host, b.descs)
    dt = (time.perf_counter() - t0) / 3
    print(f"host_batch_peso {name:9s} {dt * 1e3:8.2f} ms  {b.total_bytes / dt / GIB:6.2f} GiB/s  "
          f"match={bool((out == want).all())}", flush=True)
