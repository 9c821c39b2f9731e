"""How much of a 1.6-GB launch is fixed cost?  configs[1]'s shape (packed
1500-B segments) at 0.5, 1, 2 and 4 times its size, and the TSO shape (64-KiB
ranges) at the same byte counts, one process, interleaved rounds with the
first-timed leg rotated: t(n) = a + b * bytes, fitted per shape.  a is what
every launch pays whatever its size (the grid filling and draining the
machine); 1 / b is the rate a launch approaches as it grows.

  python scripts/launch_overhead.py [ROUNDS] [K,K,...]

With a K list, configs[1]'s shape is also timed with the packed kernel's
ranges per workgroup forced to each K (debug knob "packed"): how the fixed
cost and the rate move with the workgroup's size.
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tcp_amd as tc  # noqa: E402
from tcp_amd import workload  # noqa: E402
from tcp_amd.csum import PESO_DTYPE  # noqa: E402

SCALES = (0.5, 1, 2, 4)
N1 = 1 << 20
big = workload.make_batch("mtu", n=int(N1 * max(SCALES) * 1.03))  # room for the TSO legs
arena, descs_all = workload.materialize(big)


def per_launch(fn, reps=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


KS = [int(k) for k in sys.argv[2].split(",")] if len(sys.argv) > 2 else []


def knobbed(fn, **kn):
    def g():
        with tc.debug(**kn):
            fn()
    return g


legs = {}
for s in SCALES:
    n = int(N1 * s)
    out = torch.empty(n, dtype=torch.uint16, device="cuda")
    nbytes = n * 1500 + 26 * n
    legs[f"mtu x{s}"] = ((lambda n=n, o=out: tc.batch_peso(arena, descs_all, n, n * 1500, out=o)), nbytes)
    for K in KS:
        legs[f"mtuK{K} x{s}"] = (knobbed(legs[f"mtu x{s}"][0], packed=K), nbytes)
    L = 65536
    n64 = -(-nbytes // (L + 26))
    d = np.zeros(n64, PESO_DTYPE)
    d["offset"], d["len"], d["protocol"] = np.arange(n64, dtype=np.uint64) * np.uint64(L), L, 6
    dd = tc.descs_to_device(d)
    o64 = torch.empty(n64, dtype=torch.uint16, device="cuda")
    assert n64 * L <= arena.numel()
    legs[f"tso x{s}"] = ((lambda n64=n64, dd=dd, o=o64: tc.batch_peso(arena, dd, n64, n64 * L, out=o)), n64 * (L + 26))
for f, _ in legs.values():
    for _ in range(10):
        f()
torch.cuda.synchronize()
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 9
names = list(legs)
ts = {k: [] for k in names}
for r in range(rounds):
    for i in range(len(names)):
        k = names[(r + i) % len(names)]
        ts[k].append(per_launch(legs[k][0]))
print(f"# {rounds} rounds x 20 launches, first-timed leg rotated", flush=True)
for shape in ["mtu", "tso"] + [f"mtuK{K}" for K in KS]:
    xs, ys = [], []
    for s in SCALES:
        k = f"{shape} x{s}"
        us = float(np.median(ts[k]))
        nb = legs[k][1]
        xs.append(nb)
        ys.append(us)
        print(f"{k:11s} {nb / 1e9:7.4f} GB  {us:8.1f} us  {nb / us / 1e3:8.1f} GB/s  frac {nb / us / 1e3 / 8000:.4f}",
              flush=True)
    b, a = np.polyfit(np.array(xs), np.array(ys), 1)
    print(f"{shape}: t = {a:.2f} us + bytes / {1 / b / 1e3:.1f} GB/s  (asymptotic frac {1 / b / 1e3 / 8000:.4f}; "
          f"fixed cost {a / ys[1]:.3f} of the 1x launch)", flush=True)
