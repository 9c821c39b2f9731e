"""k_ipv4's sums kernel (32 lanes x 6 loads, the configs[3] route) in other
launch forms, against the product call: 512- / 1024-thread workgroups, and
held to 64 VGPRs (8 waves per SIMD; the route's build takes 66 VGPRs, 7
waves).  One process, interleaved rounds, median us per launch; every form's
sums must equal the product's.  tcsum_probe_ipv4_shape (libtcsum_bench.so).

  python scripts/ipv4_shape_ab.py [config ...]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tcp_amd as tc  # noqa: E402
from tcp_amd import _lib, workload  # noqa: E402

B = _lib.bench_lib()
for cfg in (sys.argv[1:] or ["mixed", "mixed_aligned"]):
    b = workload.make_batch(cfg)
    arena, descs = workload.materialize(b)
    n = b.n
    assert tc.route(b.total_bytes // n)["lanes"] == 32 and tc.route(b.total_bytes // n)["loads"] == 6
    ref, _ = tc.batch_ipv4(arena, descs, n, b.total_bytes, want_flags=False)
    ref = ref.clone()
    outs = {}

    def product(o):
        tc.batch_ipv4(arena, descs, n, b.total_bytes, out=o, want_flags=False)

    def shape(wg, occ8):
        def f(o):
            _lib.check(B.tcsum_probe_ipv4_shape(arena.data_ptr(), descs.data_ptr(), n, wg, occ8, o.data_ptr(),
                                                torch.cuda.current_stream().cuda_stream), "probe_ipv4_shape")
        return f

    kinds = {"product (k_ipv4<32,6>, 256 threads)": product, "256 threads, same kernel (probe lib)": shape(256, 0),
             "512 threads": shape(512, 0), "1024 threads": shape(1024, 0),
             "256 threads, <= 64 VGPRs (8 waves/SIMD)": shape(256, 1)}
    for k, fn in kinds.items():
        outs[k] = torch.empty(n, dtype=torch.uint32, device="cuda")
        fn(outs[k])
        torch.cuda.synchronize()
        assert torch.equal(outs[k], ref), k
    times = {k: [] for k in kinds}
    for r in range(7):
        for k, fn in kinds.items():
            fn(outs[k])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                fn(outs[k])
            e1.record()
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / 10)
    alg = b.total_bytes + 20 * n
    base = np.median(times["product (k_ipv4<32,6>, 256 threads)"])
    print(f"# {cfg}: {n} packets, {b.total_bytes} B; median of 7 rounds x 10 launches, interleaved; results equal")
    for k, t in times.items():
        m = np.median(t)
        print(f"{k:42s} {m*1e3:9.1f} us  {m/base:6.3f}x  {alg / (m*1e-3) / 8e12:6.4f} of 8 TB/s", flush=True)
    del arena, descs, outs
    torch.cuda.empty_cache()
