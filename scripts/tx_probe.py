"""Where does tx fill time go?  Interleaved rounds in one process: ipv4 sums,
tx fill (stores deferred to k_tx_scatter: the default for this size), tx fill
with the stores in the kernel (debug knob tx_split=0), tx offload (the same kernel
without the stores), rx verify.  Both fill forms must leave the same bytes.
(Round 2 also had a variant re-reading the field lines with the default cache
policy before the stores: no gain, profiles/r02/tx_probe_rx_fast.txt.)"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tcp_amd as tc  # noqa: E402
from tcp_amd import workload  # noqa: E402

b = workload.make_batch("mixed")
arena, descs = workload.materialize(b)
out = torch.empty(b.n, dtype=torch.uint32, device="cuda")
verdict = torch.empty(b.n, dtype=torch.int8, device="cuda")


def sums():
    tc.batch_ipv4(arena, descs, b.n, b.total_bytes, out=out, want_flags=False)


def tx():
    tc.batch_ipv4_tx_fill(arena, descs, b.n, b.total_bytes, want_flags=False)


def tx_fused():
    with tc.debug(tx_split=0):
        tc.batch_ipv4_tx_fill(arena, descs, b.n, b.total_bytes, want_flags=False)


outo = torch.empty(b.n, dtype=torch.uint32, device="cuda")
flo = torch.empty(b.n, dtype=torch.uint8, device="cuda")


def tx_offload():
    tc.batch_ipv4_tx_offload(arena, descs, b.n, b.total_bytes, out=outo, flags=flo)


def rx():
    tc.batch_ipv4_rx_verify(arena, descs, b.n, b.total_bytes, verdict=verdict, want_flags=False)


tx()
ref = arena.clone()
tx_fused()
assert torch.equal(arena, ref), "the two fill forms left different bytes"
variants = {"sums": sums, "tx": tx, "tx_fused": tx_fused, "tx_offload": tx_offload, "rx": rx}
times = {k: [] for k in variants}
for r in range(5):
    for k, fn in variants.items():
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        times[k].append(e0.elapsed_time(e1) / 10)
for k, t in times.items():
    print(f"{k:12s} {np.median(t)*1e3:8.1f} us")
