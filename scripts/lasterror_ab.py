"""Round 4's intermittent TCSUM_ERR_SYS, before and after (profiles/history/DESIGN_rounds1-5.md §5):
one process, two builds of libtcsum.so -- round 4's (launches judged by the
thread's last-error slot) and this tree's (each launch's own status) -- each
called right after the calling thread's slot was left dirty, by a NotReady
poll of a busy stream and by a failed call of the caller's own.

  python scripts/lasterror_ab.py abl/libtcsum_r04.so tcp_amd/libtcsum.so
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tcp_amd as tc  # noqa: E402
from tcp_amd import _lib, workload  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so.7")
hip.hipStreamQuery.argtypes = [ctypes.c_void_p]
hip.hipSetDevice.argtypes = [ctypes.c_int]


def load(path):
    L = ctypes.CDLL(os.path.abspath(path))
    for name, (res, args) in _lib.SIGNATURES.items():
        f = getattr(L, name, None)
        if f is not None:
            f.restype, f.argtypes = res, args
    return L


def dirty(kind):
    if kind == "not_ready":
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            torch.cuda._sleep(50_000_000)
        q = hip.hipStreamQuery(ctypes.c_void_p(s.cuda_stream))
        slot = hip.hipPeekAtLastError()
        s.synchronize()
        return f"hipStreamQuery -> {q}, slot {slot}"
    n = ctypes.c_int(0)
    hip.hipGetDeviceCount(ctypes.byref(n))
    r = hip.hipSetDevice(n.value)
    hip.hipSetDevice(0)
    return f"hipSetDevice({n.value}) -> {r}, slot {hip.hipPeekAtLastError()}"


b = workload.make_batch("mtu", n=4096)
arena, descs = workload.materialize(b)
want = tc.batch_peso(arena, descs, b.n, b.total_bytes).cpu().numpy()
host = arena.cpu().numpy()
for path in sys.argv[1:]:
    L = load(path)
    for kind in ("not_ready", "invalid_device"):
        for call in ("tcsum_batch_peso", "tcsum_host_batch_peso"):
            hip.hipGetLastError()
            out = torch.zeros(b.n, dtype=torch.uint16, device="cuda")
            ho = np.zeros(b.n, np.uint16)
            torch.cuda.synchronize()
            how = dirty(kind)
            if call == "tcsum_batch_peso":
                rc = L.tcsum_batch_peso(arena.data_ptr(), descs.data_ptr(), b.n, out.data_ptr(), b.total_bytes,
                                        torch.cuda.current_stream().cuda_stream)
            else:
                rc = L.tcsum_host_batch_peso(0, host.ctypes.data, host.nbytes, b.descs.ctypes.data, b.n,
                                             ho.ctypes.data)
            left = hip.hipGetLastError()  # what the call left in the slot (then cleared for torch's own checks)
            torch.cuda.synchronize()
            same = bool(((out.cpu().numpy() if call == "tcsum_batch_peso" else ho) == want).all())
            how += f"; slot after the call {left}"
            print(f"{os.path.basename(path):22s} {kind:15s} ({how}) {call:22s} rc {rc:3d} results "
                  f"{'equal' if same else 'NOT equal'}", flush=True)
    hip.hipGetLastError()
