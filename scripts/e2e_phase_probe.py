"""Where the end-to-end host batch loses to a plain H2D copy (configs[1]):
the copy of the same bytes, the descriptors' own copy, the fixed cost of a
small call, and one traced call (debug knob e2e_trace: host-side phase times).
Measurement script, not product code; run it under rocprofv3
--memory-copy-trace --kernel-trace for the device side."""
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
del arena
torch.cuda.empty_cache()


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


pinned = torch.from_numpy(host)
dst = torch.empty(b.alloc_bytes, dtype=torch.uint8, device="cuda")
dt = timed(lambda: dst.copy_(pinned, non_blocking=True))
print(f"plain H2D copy of the arena      {dt * 1e3:8.3f} ms  {b.alloc_bytes / dt / GIB:7.2f} GiB/s", flush=True)
del dst
dbytes = b.descs.nbytes
pd = L.tcsum_host_alloc(dbytes)
hd = np.ctypeslib.as_array((ctypes.c_uint8 * dbytes).from_address(pd))
hd[:] = b.descs.view(np.uint8).reshape(-1)
ddst = torch.empty(dbytes, dtype=torch.uint8, device="cuda")
dt = timed(lambda: ddst.copy_(torch.from_numpy(hd), non_blocking=True), 10)
print(f"plain H2D copy of the descriptors {dt * 1e3:7.3f} ms  ({dbytes / 1e6:.1f} MB)", flush=True)
res = torch.empty(b.n, dtype=torch.uint16, device="cuda")
hres = np.empty(b.n, np.uint16)
dt = timed(lambda: hres.__setitem__(slice(None), res.cpu().numpy()), 10)
print(f"D2H of the results (pageable)     {dt * 1e3:7.3f} ms", flush=True)
out = tc.host_batch_peso(host, b.descs)
dt = timed(lambda: tc.host_batch_peso(host, b.descs))
print(f"host_batch_peso (full)           {dt * 1e3:8.3f} ms  {b.total_bytes / dt / GIB:7.2f} GiB/s  "
      f"match={bool((out == want).all())}", flush=True)
small = b.descs[:4096]
dt = timed(lambda: tc.host_batch_peso(host, small), 20)
print(f"host_batch_peso (4096 segments)  {dt * 1e3:8.3f} ms  (fixed cost of a call)", flush=True)
tc.debug_set("e2e_trace", 1)
print("traced full call (host-side phases on stderr):", flush=True)
tc.host_batch_peso(host, b.descs)
L.tcsum_host_free(pd)
L.tcsum_host_free(p)
