"""tcsum_host_batch_peso from pinned host memory (configs[1], PCIe-inclusive),
two or more builds of libtcsum.so in one process, interleaved rounds with the
build timed first rotated, plus the plain pinned -> device copy of the same
bytes each round.  Round 5's default line read 48.7 GiB/s where rounds 3-4
read 51.5: this tells a library change from a box.

  python scripts/e2e_ab.py abl/libtcsum_r04.so tcp_amd/libtcsum.so [--rounds N]
"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tcp_amd as tc  # noqa: E402
from tcp_amd import _lib, workload  # noqa: E402

GIB = 1 << 30


def load(path):
    L = ctypes.CDLL(os.path.abspath(path))
    for name, (res, args) in _lib.SIGNATURES.items():
        f = getattr(L, name, None)
        if f is not None:
            f.restype, f.argtypes = res, args
    return L


args = [a for a in sys.argv[1:] if not a.startswith("--")]
rounds = int(sys.argv[sys.argv.index("--rounds") + 1]) if "--rounds" in sys.argv else 7
args = [a for a in args if not a.isdigit()]
b = workload.make_batch("mtu")
arena, descs = workload.materialize(b)
want = tc.batch_peso(arena, descs, b.n, b.total_bytes).cpu().numpy()
P = _lib.lib()
p = P.tcsum_host_alloc(b.alloc_bytes)
host = np.ctypeslib.as_array((ctypes.c_uint8 * b.alloc_bytes).from_address(p))
host[:] = arena[: b.alloc_bytes].cpu().numpy()
segs = np.ascontiguousarray(b.descs)
del arena, descs
torch.cuda.empty_cache()
libs = {os.path.basename(a) if a.count("/") < 2 else a: load(a) for a in args}
out = {k: np.zeros(b.n, np.uint16) for k in libs}


def run(L, o):
    rc = L.tcsum_host_batch_peso(0, host.ctypes.data, host.nbytes, segs.ctypes.data, b.n, o.ctypes.data)
    assert rc == 0, rc


pinned = torch.from_numpy(host)
dst = torch.empty(b.alloc_bytes, dtype=torch.uint8, device="cuda")


def copy():
    dst.copy_(pinned, non_blocking=True)
    torch.cuda.synchronize()


legs = {"plain H2D copy": copy}
for k, L in libs.items():
    legs[k] = (lambda L=L, o=out[k]: run(L, o))
for f in legs.values():
    f()
    f()
names = list(legs)
ts = {k: [] for k in names}
for r in range(rounds):
    for i in range(len(names)):
        k = names[(r + i) % len(names)]
        t0 = time.perf_counter()
        for _ in range(3):
            legs[k]()
        ts[k].append((time.perf_counter() - t0) / 3)
print(f"# configs[1] from pinned host memory; {rounds} rounds x 3 calls, first-timed leg rotated", flush=True)
for k in names:
    nb = b.alloc_bytes if k == "plain H2D copy" else b.total_bytes
    med = float(np.median(ts[k]))
    ok = "" if k == "plain H2D copy" else f"  results {'equal' if (out[k] == want).all() else 'NOT equal'}"
    print(f"{k:28s} {med * 1e3:8.2f} ms  {nb / med / GIB:7.2f} GiB/s  (best {nb / min(ts[k]) / GIB:.2f}){ok}",
          flush=True)
P.tcsum_host_free(p)
