"""Does a host-memory batch slow the device-resident kernels that follow it?

One process: configs[2] (16 GiB, device-resident) timed, then bench.py's e2e
leg (tcsum_host_batch_peso from a pinned arena of the configs[1] batch) and
the drop-in calls, then configs[2] again, then after tcsum_release(0), then
after a 2-s pause.  Median us per launch of 7 rounds x 10 launches each time.

  python scripts/after_host_batch.py
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import tcp_amd as tc  # noqa: E402
from tcp_amd import workload  # noqa: E402


def timed(b, arena, descs, out):
    ts = []
    for _ in range(7):
        tc.batch_peso(arena, descs, b.n, b.total_bytes, out=out)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            tc.batch_peso(arena, descs, b.n, b.total_bytes, out=out)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 10 * 1e3)
    return float(np.median(ts))


tso = workload.make_batch("tso")
a, d = workload.materialize(tso)
o = torch.empty(tso.n, dtype=torch.uint16, device="cuda")
print(f"tso first                      {timed(tso, a, d, o):9.1f} us", flush=True)
head = bench.time_config(torch, tc, workload, "mtu", 0, 20, 10, probes=False)
print(f"tso after an mtu batch         {timed(tso, a, d, o):9.1f} us", flush=True)
e = bench.e2e(torch, tc, head)
print(f"  (e2e leg: {e.get('gib_s')} GiB/s)", flush=True)
print(f"tso after the e2e leg          {timed(tso, a, d, o):9.1f} us", flush=True)
bench.legacy_latency(tc)
print(f"tso after the drop-in calls    {timed(tso, a, d, o):9.1f} us", flush=True)
tc.release(0)
print(f"tso after tcsum_release(0)     {timed(tso, a, d, o):9.1f} us", flush=True)
time.sleep(2)
print(f"tso after a 2-s pause          {timed(tso, a, d, o):9.1f} us", flush=True)
del head
torch.cuda.empty_cache()
print(f"tso after freeing the mtu batch {timed(tso, a, d, o):9.1f} us", flush=True)
