"""Price the byte-window stream's pieces on configs[3] (ONE process,
interleaved rounds, median us per launch): the product's per-packet kernel
(k_ipv4), the stream in several workgroup shapes, and its probe forms
(tcsum_probe_flat: 1 = plan + window loads, 2 = + LDS prefix scans, 3 = all
but the cross-window combine, 0 = the full stream's sums).

  python scripts/flat_probe.py [config] [shapes, e.g. 4x3,16x4]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tcp_amd as tc  # noqa: E402
from tcp_amd import _lib, workload  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "mixed"
shapes = [tuple(map(int, s.split("x"))) for s in (sys.argv[2] if len(sys.argv) > 2 else "4x3,8x3,8x4,16x4,16x2").split(",")]
b = workload.make_batch(cfg)
arena, descs = workload.materialize(b)
n = b.n
out = torch.empty(n, dtype=torch.uint32, device="cuda")
sink = torch.zeros(1, dtype=torch.uint32, device="cuda")
B = _lib.bench_lib()
ref, _ = tc.batch_ipv4(arena, descs, n, b.total_bytes, want_flags=False)
ref = ref.clone()


def product():
    tc.batch_ipv4(arena, descs, n, b.total_bytes, out=out, want_flags=False)


def product_flat():
    with tc.debug(flat=1):
        tc.batch_ipv4(arena, descs, n, b.total_bytes, out=out, want_flags=False)


def probe(variant, w, u):
    def f():
        o = out if variant in (0, 3) else sink  # variants 0 and 3 write out[0..n): a 1-word sink would overflow
        _lib.check(B.tcsum_probe_flat(arena.data_ptr(), descs.data_ptr(), n, b.total_bytes, variant, w, u,
                                      o.data_ptr(), o.numel(), None, torch.cuda.current_stream().cuda_stream),
                   "probe_flat")
    return f


kinds = {"k_ipv4 (product default)": product, "flat 4x3 (product, knob)": product_flat,
         "plain read probe": lambda: tc.probe_read(arena, b.arena_bytes, sink)}
for w, u in shapes:
    for v in (0, 1, 2, 3):
        kinds[f"flat {w}x{u} v{v}"] = probe(v, w, u)
# the variants that compute real sums must equal the product's
for name in ["flat 4x3 (product, knob)"] + [f"flat {w}x{u} v0" for w, u in shapes]:
    out.zero_()
    kinds[name]()
    torch.cuda.synchronize()
    assert torch.equal(out, ref), name
times = {k: [] for k in kinds}
for r in range(7):
    for k, fn in kinds.items():
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        times[k].append(e0.elapsed_time(e1) / 10)
alg = b.total_bytes + 20 * n
base = np.median(times["k_ipv4 (product default)"])
print(f"# {cfg}: {n} packets, {b.total_bytes} B; median of 7 rounds x 10 launches, interleaved")
for k, t in times.items():
    m = np.median(t)
    print(f"{k:32s} {m*1e3:9.1f} us  {m/base:6.3f}x  {alg / (m*1e-3) / 8e12:6.4f} of 8 TB/s")
