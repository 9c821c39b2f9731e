"""Price the byte-window stream's pieces on configs[3] (ONE process,
interleaved rounds, median us per launch): the product's per-packet kernel
(k_ipv4), the stream in several workgroup shapes, and its probe forms
(tcsum_probe_flat: 1 = plan + window loads, 2 = + LDS prefix scans, 3 = all
but the cross-window combine, 0 = the full stream's sums).

  python scripts/flat_probe.py [config] [shapes, e.g. 4x3,16x4] [variants, e.g. 0,1] [extra]

extra: also the packet-agnostic ceiling on the same arena (its bytes cut into
64-KiB checksum_peso ranges: the TSO kernel, k_segments_wgx<16,32,4>), the
product's tile-shaped read probes, and k_ipv4 in its other compiled shapes
(debug lanes x loads).
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
variants = [int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "0,1,2,3").split(",")]
extra = len(sys.argv) > 4 and sys.argv[4] == "extra"
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


def product_flat():  # round 4's route candidate, libtcsum_bench.so since round 5
    tc.flat_ipv4(0, arena, descs, n, b.total_bytes, out=out)


def probe(variant, w, u):
    def f():
        o = out if variant in (0, 3) else sink  # variants 0 and 3 write out[0..n): a 1-word sink would overflow
        _lib.check(B.tcsum_probe_flat(arena.data_ptr(), descs.data_ptr(), n, b.total_bytes, variant, w, u,
                                      o.data_ptr(), o.numel(), None, torch.cuda.current_stream().cuda_stream),
                   "probe_flat")
    return f


kinds = {"k_ipv4 (product default)": product, "flat 4x3 (tcsum_flat_ipv4)": product_flat,
         "plain read probe": lambda: tc.probe_read(arena, b.arena_bytes, sink)}
for w, u in shapes:
    for v in variants:
        kinds[f"flat {w}x{u} v{v}"] = probe(v, w, u)
if extra:
    from tcp_amd.csum import PESO_DTYPE
    L64 = 65536
    n64 = b.arena_bytes // L64
    p64 = np.zeros(n64, PESO_DTYPE)
    p64["offset"] = np.arange(n64, dtype=np.uint64) * np.uint64(L64)
    p64["len"] = L64
    p64["protocol"] = 6
    d64 = tc.descs_to_device(p64)
    o64 = torch.empty(n64, dtype=torch.uint16, device="cuda")
    kinds["64-KiB ranges (wgx<16,32,4>)"] = lambda: tc.batch_peso(arena, d64, n64, n64 * L64, out=o64)
    for g, u, dep in ((32, 4, True), (32, 6, True), (64, 4, False), (256, 4, False)):
        kinds[f"tile {g}x{u}{' dep' if dep else ''}"] = (
            lambda g=g, u=u, dep=dep: tc.probe_tile(arena, b.arena_bytes, g, u, sink, dep=dep))
    for g, u in ((64, 4), (16, 8), (64, 16)):
        def shaped(g=g, u=u):
            with tc.debug(lanes=g, loads=u):
                tc.batch_ipv4(arena, descs, n, b.total_bytes, out=out, want_flags=False)
        kinds[f"k_ipv4 {g}x{u} (knob)"] = shaped
# the variants that compute real sums must equal the product's
for name in ["flat 4x3 (tcsum_flat_ipv4)"] + [f"flat {w}x{u} v0" for w, u in shapes if 0 in variants] + \
        [k for k in kinds if k.startswith("k_ipv4 ") and "knob" in k]:
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
