"""End-to-end (PCIe-inclusive) rate of tcsum_host_batch_peso on configs[1]
by copy-chunk size, next to the plain pinned H2D copy rate of the same bytes
(torch non_blocking copy, one shot).  Measurement script, not product code."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tcp_amd as tc  # noqa: E402
from tcp_amd import _lib, workload  # noqa: E402

GIB = 1 << 30
b = workload.make_batch("mtu")
arena, descs = workload.materialize(b)
want = tc.batch_peso(arena, descs, b.n, b.total_bytes).cpu().numpy()
L = _lib.lib()
p = L.tcsum_host_alloc(b.alloc_bytes)
host = np.ctypeslib.as_array((ctypes.c_uint8 * b.alloc_bytes).from_address(p))
host[:] = arena[: b.alloc_bytes].cpu().numpy()

# plain copy engine rate, pinned -> device, same bytes
pinned = torch.from_numpy(host)  # memory is pinned by hipHostMalloc
dst = torch.empty(b.alloc_bytes, dtype=torch.uint8, device="cuda")
for _ in range(2):
    dst.copy_(pinned, non_blocking=True)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5):
    dst.copy_(pinned, non_blocking=True)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 5
print(f"plain H2D copy (one shot)        {b.alloc_bytes / dt / GIB:7.2f} GiB/s", flush=True)

for mb in (None, 32, 64, 128, 256, 384, 512):
    if mb is None:  # the library's own choice (a quarter of the batch, >= 64 MiB)
        tc.debug_set("e2e_chunk_mb", -1)
    else:
        tc.debug_set("e2e_chunk_mb", mb)
    out = tc.host_batch_peso(host, b.descs)
    t0 = time.perf_counter()
    for _ in range(5):
        out = tc.host_batch_peso(host, b.descs)
    dt = (time.perf_counter() - t0) / 5
    ok = bool((out == want).all())
    label = "default" if mb is None else f"{mb:4d} MiB"
    print(f"host_batch_peso chunk {label:>8}     {b.total_bytes / dt / GIB:7.2f} GiB/s  match={ok}", flush=True)
L.tcsum_host_free(p)
