"""tx fill called the way a host loop calls it: one fill, then a stream sync,
repeated (wall time per call).  The deferred form allocates its scratch with
stream-ordered allocation on every call; this shows what that costs when every
call is synchronized (the pool may hand memory back between calls), against
the fill with its stores in the kernel, for configs[3] and smaller batches."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tcp_amd as tc  # noqa: E402
from tcp_amd import workload  # noqa: E402

for n in (131072, 1 << 20):
    b = workload.make_batch("mixed_tx", n=n)
    arena, descs = workload.materialize(b)
    res = {}
    for split in ("0", "1"):
        tc.debug_set("tx_split", int(split))
        for _ in range(3):
            tc.batch_ipv4_tx_fill(arena, descs, b.n, b.total_bytes, want_flags=False)
        torch.cuda.synchronize()
        ts = []
        for _ in range(30):
            t0 = time.perf_counter()
            tc.batch_ipv4_tx_fill(arena, descs, b.n, b.total_bytes, want_flags=False)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        res[split] = np.median(ts) * 1e6
    tc.debug_set("tx_split", -1)
    print(f"n {n:8d}: fused {res['0']:8.1f} us   deferred {res['1']:8.1f} us per synchronized call", flush=True)
    del arena, descs
    torch.cuda.empty_cache()
