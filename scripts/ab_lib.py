"""A/B two or more builds of libtcsum.so in ONE process (box-to-box spread is
larger than the effects measured): interleaved rounds whose starting build
rotates (the first build timed in a round measured ~1 % slow on the headline,
whichever it was), median ms per launch, and the outputs of every build must
be identical (AB_ALLOW_DIFF=1 for measurement builds that store nothing).

  python scripts/ab_lib.py LIB_A LIB_B [LIB_C ...] [configs]
  (configs: mtu,tso,mixed,mixed_tx,mixed_rx; uNNNN / uNNNN_rx / uNNNN_tx:
  IPv4 packets of NNNN bytes each, as many as configs[3]'s bytes hold)
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tcp_amd as tc  # noqa: E402
from tcp_amd import _lib, workload  # noqa: E402


def load(path):
    L = ctypes.CDLL(os.path.abspath(path))
    for name, (res, args) in _lib.SIGNATURES.items():
        f = getattr(L, name, None)  # an older build may lack newer symbols
        if f is not None:
            f.restype, f.argtypes = res, args
    return L


paths = [a for a in sys.argv[1:] if a.endswith(".so")]
rest = [a for a in sys.argv[1:] if not a.endswith(".so")]
libs = [load(p) for p in paths]
configs = rest[0].split(",") if rest else ["mtu", "tso", "mixed", "mixed_tx", "mixed_rx"]
rounds, reps = 8, 10
def equal_length(L):
    from tcp_amd.csum import PKT_DTYPE
    total = workload.make_batch("mixed").total_bytes
    n = total // L
    d = np.zeros(n, PKT_DTYPE)
    d["offset"] = np.arange(n, dtype=np.uint64) * np.uint64(L)
    d["len"] = L
    return workload.Batch("mixed", "ipv4", n, d, n * L, n * L, 0, op="sums")


for cfg in configs:
    label = cfg
    if cfg.startswith("u"):
        b = equal_length(int(cfg[1:].split("_")[0]))
        cfg = "mixed" + cfg[len(cfg.split("_")[0]):]
    else:
        base = cfg.split("_")[0] if cfg in ("mixed_tx", "mixed_rx") else cfg
        b = workload.make_batch(base)
    arena, descs = workload.materialize(b)
    peso = b.kind == "peso"
    outs = [torch.empty(b.n, dtype=torch.uint16 if peso else torch.uint32, device="cuda") for _ in libs]
    verdicts = [torch.zeros(b.n, dtype=torch.int8, device="cuda") for _ in libs]
    if cfg == "mixed_tx":  # fill once: every timed launch rewrites the same values
        tc.batch_ipv4_tx_fill(arena, descs, b.n, b.total_bytes, want_flags=False)

    def run(i):
        _lib._lib = libs[i]
        if peso:
            tc.batch_peso(arena, descs, b.n, b.total_bytes, out=outs[i])
        elif cfg == "mixed_tx":
            tc.batch_ipv4_tx_fill(arena, descs, b.n, b.total_bytes, out=outs[i], want_flags=False)
        elif cfg == "mixed_rx":
            tc.batch_ipv4_rx_verify(arena, descs, b.n, b.total_bytes, verdict=verdicts[i], out=outs[i],
                                    want_flags=False)
        else:
            tc.batch_ipv4(arena, descs, b.n, b.total_bytes, out=outs[i], want_flags=False)

    times = [[] for _ in libs]
    for r in range(rounds):
        for k in range(len(libs)):
            i = (r + k) % len(libs)
            run(i)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                run(i)
            e1.record()
            torch.cuda.synchronize()
            times[i].append(e0.elapsed_time(e1) / reps)
    same = all(torch.equal(outs[0], o) for o in outs[1:]) and all(torch.equal(verdicts[0], v) for v in verdicts[1:])
    print(f"== {label} n={b.n} bytes={b.total_bytes} identical={same}", flush=True)
    for i, p in enumerate(paths):
        med = float(np.median(times[i]))
        print(f"  {os.path.basename(p):24s} {med * 1e3:8.1f} us  {b.total_bytes / med / 1e6:8.1f} GB/s payload"
              f"  (min {min(times[i]) * 1e3:.1f})", flush=True)
    assert same or os.environ.get("AB_ALLOW_DIFF") == "1", cfg
    del arena, descs, outs
    torch.cuda.empty_cache()
