"""A/B of two libtcsum.so builds on the host-memory batches, in ONE process
(interleaved rounds, median wall time per call): host-queue rx verify and tx
fill (pinned / pageable) and the bulk host_batch_peso.  Every build's results
must match.  Measurement script, not product code.

  python scripts/hostq_ab.py LIB_A LIB_B [n_frames]
"""
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
paths = sys.argv[1:3]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 20


def load(path):
    L = ctypes.CDLL(os.path.abspath(path))
    for name, (res, args) in _lib.SIGNATURES.items():
        f = getattr(L, name, None)
        if f is not None:
            f.restype, f.argtypes = res, args
    return L


libs = [load(p) for p in paths]
b = workload.make_batch("mixed_tx", n=n)
arena, descs = workload.materialize(b)
raw = arena.cpu().numpy()
del arena, descs
ha = tc.HostArena(raw.size)
ha.array[:] = raw
page = raw.copy()
m = workload.make_batch("mtu")
marena, mdescs = workload.materialize(m)
mhost = tc.HostArena(m.alloc_bytes)
mhost.array[:] = marena[: m.alloc_bytes].cpu().numpy()
del marena, mdescs
torch.cuda.empty_cache()
cases = {
    "rx pinned": (lambda: tc.host_batch_ipv4_rx_verify(ha, b.descs), b.total_bytes),
    "rx pageable": (lambda: tc.host_batch_ipv4_rx_verify(page, b.descs), b.total_bytes),
    "tx pinned": (lambda: tc.host_batch_ipv4_tx_fill(ha, b.descs), b.total_bytes),
    "tx pageable": (lambda: tc.host_batch_ipv4_tx_fill(page, b.descs), b.total_bytes),
    "peso e2e": (lambda: tc.host_batch_peso(mhost.array, m.descs), m.total_bytes),
}
res = {k: [[] for _ in libs] for k in cases}
outs = {k: [None for _ in libs] for k in cases}
for r in range(5):
    for k, (fn, nbytes) in cases.items():
        for j in (range(len(libs)) if r % 2 == 0 else reversed(range(len(libs)))):
            _lib._lib = libs[j]
            o = fn()
            t0 = time.perf_counter()
            o = fn()
            res[k][j].append(time.perf_counter() - t0)
            first = o[0] if isinstance(o, tuple) else o
            outs[k][j] = np.asarray(first).copy()
print(f"# {n} mixed frames ({b.total_bytes} B); peso e2e: configs[1] ({m.total_bytes} B); median of 5 rounds")
for k, (fn, nbytes) in cases.items():
    same = all(np.array_equal(outs[k][0], o) for o in outs[k][1:])
    line = "  ".join(f"{os.path.basename(p)} {np.median(res[k][j]) * 1e3:8.2f} ms {nbytes / np.median(res[k][j]) / GIB:6.2f} GiB/s"
                     for j, p in enumerate(paths))
    print(f"{k:12s} {line}  same={same}", flush=True)
