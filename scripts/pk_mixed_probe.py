"""Could configs[3] gain from the packed stream?  Its 1M IPv4 packets
(64..9000 B, packed) summed as checksum_peso ranges -- the arithmetic the
IPv4 kernel does minus the header parsing -- by the per-range kernel and by
k_segments_pk in several shapes, next to tcsum_batch_ipv4 on the same bytes.
One process, interleaved rounds, median us per launch.

  python scripts/pk_mixed_probe.py
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tcp_amd as tc  # noqa: E402
from tcp_amd import workload  # noqa: E402
from tcp_amd.csum import PESO_DTYPE  # noqa: E402

b = workload.make_batch("mixed")
arena, descs = workload.materialize(b)
p = np.zeros(b.n, PESO_DTYPE)
p["offset"], p["len"] = b.descs["offset"], b.descs["len"]
p["protocol"] = 6
dp = tc.descs_to_device(p)
o16 = torch.empty(b.n, dtype=torch.uint16, device="cuda")
o32 = torch.empty(b.n, dtype=torch.uint32, device="cuda")
nbytes = b.total_bytes + 26 * b.n


def env(e):
    def set_():
        for k in ("TCSUM_PACKED", "TCSUM_PK_W", "TCSUM_PK_U"):
            os.environ.pop(k, None)
        os.environ.update(e)
    return set_


legs = {
    "ipv4 sums (k_ipv4)": (env({}), lambda: tc.batch_ipv4(arena, descs, b.n, b.total_bytes, out=o32, want_flags=False)),
    "peso per-range": (env({"TCSUM_PACKED": "0"}), lambda: tc.batch_peso(arena, dp, b.n, b.total_bytes, out=o16)),
}
for w, u in ((4, 3), (8, 3), (16, 2)):
    legs[f"peso packed W{w} U{u}"] = (env({"TCSUM_PACKED": "1", "TCSUM_PK_W": str(w), "TCSUM_PK_U": str(u)}),
                                      lambda: tc.batch_peso(arena, dp, b.n, b.total_bytes, out=o16))
# the same bytes cut into 64-KiB ranges: the TSO kernel's stream (the ceiling a
# packet-agnostic load shape reaches on this arena)
L64 = 65536
n64 = b.arena_bytes // L64
p64 = np.zeros(n64, PESO_DTYPE)
p64["offset"] = np.arange(n64, dtype=np.uint64) * np.uint64(L64)
p64["len"] = L64
p64["protocol"] = 6
d64 = tc.descs_to_device(p64)
o64 = torch.empty(n64, dtype=torch.uint16, device="cuda")
legs["as 64-KiB ranges (wgx)"] = (env({}), lambda: tc.batch_peso(arena, d64, n64, n64 * L64, out=o64))
ref = None
ts = {k: [] for k in legs}
for r in range(8):
    for k, (setup, fn) in legs.items():
        setup()
        fn()
        torch.cuda.synchronize()
        if k.startswith("peso "):
            if ref is None:
                ref = o16.clone()
            assert torch.equal(o16, ref), k
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        if r:
            ts[k].append(e0.elapsed_time(e1) / 10 * 1e3)
env({})()
for k in legs:
    us = float(np.median(ts[k]))
    print(f"{k:24s} {us:8.1f} us  {nbytes / us / 1e3 / 8000:.4f} of spec", flush=True)
