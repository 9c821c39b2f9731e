"""Host-queue IPv4 batches: latency / throughput of tx fill and rx verify on
frames in host memory, pinned (kernel reads/writes in place over PCIe) vs
pageable (staged).  Prints one line per (n, memory, op)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tcp_amd as tc  # noqa: E402
from tcp_amd import workload  # noqa: E402

tc.plat_init(0)
if os.environ.get("TCSUM_PROBE_SERVER") == "1":  # serve the calls from the resident grid
    tc.queue_server(True)
sizes = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [1, 50, 1024, 65536, 1 << 20]
for n in sizes:
    b = workload.make_batch("mixed_tx", n=n)
    arena, descs = workload.materialize(b)
    raw = arena.cpu().numpy()
    del arena, descs
    ha = tc.HostArena(raw.size)
    ha.array[:] = raw
    page = raw.copy()
    reps = 200 if n <= 1024 else 20 if n <= 65536 else 5
    for mem, arg in (("pinned", ha), ("pageable", page)):
        for op in ("tx", "rx"):
            f = (lambda: tc.host_batch_ipv4_tx_fill(arg, b.descs)) if op == "tx" else \
                (lambda: tc.host_batch_ipv4_rx_verify(arg, b.descs))
            f()
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                f()
                ts.append(time.perf_counter() - t0)
            t = float(np.median(ts))
            print(f"n={n:8d} {mem:8s} {op}: {t*1e6:10.1f} us/call  {b.total_bytes/t/2**30:8.2f} GiB/s"
                  f"  ({b.total_bytes} B)", flush=True)
    ha.free()
if os.environ.get("TCSUM_PROBE_SERVER") == "1":
    tc.queue_server(False)  # debug knob server_trace=1: prints the grid's phase timings
