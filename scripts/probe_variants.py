"""The read probe's own variants (loads per lane, cache policy, XCD order) on
the configs[1] and configs[2] bytes, interleaved rounds in one process: is
bench.py's "achievable" read the best plain read?  (measurement script)"""
import itertools
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tcp_amd as tc  # noqa: E402
from tcp_amd import workload  # noqa: E402

for cfg in ("mtu", "tso"):
    b = workload.make_batch(cfg)
    arena, descs = workload.materialize(b)
    sink = torch.zeros(1, dtype=torch.uint32, device="cuda")
    variants = list(itertools.product((4, 8, 16), (1, 0), (1, 64)))
    times = {v: [] for v in variants}
    for r in range(5):
        for v in variants:
            os.environ["TCSUM_PROBE_U"], os.environ["TCSUM_PROBE_NT"], os.environ["TCSUM_PROBE_XCD"] = map(str, v)
            tc.probe_read(arena, b.arena_bytes, sink)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                tc.probe_read(arena, b.arena_bytes, sink)
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / 10)
    print(f"== {cfg} bytes={b.arena_bytes}", flush=True)
    for v in sorted(variants, key=lambda v: np.median(times[v])):
        us = np.median(times[v]) * 1e3
        print(f"  U={v[0]:2d} nt={v[1]} xcd={v[2]:3d}  {us:9.1f} us  {b.arena_bytes / us / 1e3:8.1f} GB/s", flush=True)
    del arena, descs
    torch.cuda.empty_cache()
