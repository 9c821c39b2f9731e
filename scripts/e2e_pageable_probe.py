"""tcsum_host_batch_peso on configs[1] from a pinned arena (tcsum_host_alloc)
and from a pageable numpy array, same bytes, one process; descriptors in
offset order and shuffled (a shuffled batch collapses to one chunk, the whole
span), the pageable arena through the library's pinned slots (default) and
through the runtime's own pageable copy (debug knob page_stage = 0).
Interleaved rounds; every result equal to the device-resident batch's.
Measurement script, not product code.

  python scripts/e2e_pageable_probe.py [ROUNDS]
"""
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
want = tc.to_host(tc.batch_peso(arena, descs, b.n, b.total_bytes))
ha = tc.HostArena(b.alloc_bytes)
ha.array[:] = tc.to_host(arena[: b.alloc_bytes])
page = np.array(ha.array)
del arena, descs
torch.cuda.empty_cache()
perm = np.random.default_rng(5).permutation(b.n)
shuf = np.ascontiguousarray(b.descs[perm])
legs = {
    "pinned, ordered": (ha.array, b.descs, None, want),
    "pageable, ordered": (page, b.descs, None, want),
    "pinned, shuffled": (ha.array, shuf, None, want[perm]),
    "pageable, shuffled": (page, shuf, None, want[perm]),
    "pageable, shuffled, page_stage=0": (page, shuf, 0, want[perm]),
    "pageable, ordered, page_stage=0": (page, b.descs, 0, want),
}
ts = {k: [] for k in legs}
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
names = list(legs)
for r in range(rounds):
    for i in range(len(names)):
        k = names[(r + i) % len(names)]
        host, d, ps, w = legs[k]
        with tc.debug(page_stage=ps):
            out = tc.host_batch_peso(host, d)
            assert (out == w).all(), k
            t0 = time.perf_counter()
            for _ in range(3):
                tc.host_batch_peso(host, d)
            ts[k].append((time.perf_counter() - t0) / 3)
print(f"# configs[1] (1M x 1500 B, {b.total_bytes / 1e9:.2f} GB) host -> GPU -> host, median of {rounds} "
      "interleaved rounds x 3 calls; results equal", flush=True)
for k in names:
    dt = float(np.median(ts[k]))
    print(f"host_batch_peso {k:34s} {dt * 1e3:8.2f} ms  {b.total_bytes / dt / GIB:6.2f} GiB/s", flush=True)
