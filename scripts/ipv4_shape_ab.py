"""k_ipv4 (the configs[3] route: sums 32 lanes x 6 loads, rx 16 x 6) in
launch forms the route does not take, against the product call: 512- /
1024-thread workgroups, and held to 7 / 8 waves per SIMD (the route's builds
take sums 66 VGPRs = 7 waves, rx 74 = 6).  One process, interleaved rounds,
median us per launch; every form's results must equal the product's.
tcsum_probe_ipv4_shape (libtcsum_bench.so).

  python scripts/ipv4_shape_ab.py [config ...]   (mixed, mixed_aligned: sums; mixed_rx: rx verify;
                                                 uNNNN / uNNNN_rx: every packet NNNN B)
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tcp_amd as tc  # noqa: E402
from tcp_amd import _lib, workload  # noqa: E402

B = _lib.bench_lib()
SKEW_ONLY = "--skew" in sys.argv
DB_ONLY = "--db" in sys.argv  # two data passes in flight, with and without the descriptor prefetch
DYN_ONLY = "--dyn" in sys.argv  # packets handed out inside the workgroup (k_ipv4_dyn), M per lane group
ROLL_ONLY = "--roll" in sys.argv  # rolling load slots: a multi-pass packet keeps its loads in flight
HDRX_ONLY = "--hdrx" in sys.argv  # header chunks shuffled from the first data pass instead of loaded
SDESC_ONLY = "--sdesc" in sys.argv  # the descriptors by scalar loads
LDS_ONLY = "--lds" in sys.argv  # later passes by LDS-DMA into a per-wave ring (PIPE 5); the 3rd header chunk as a dword
SMALLWG_ONLY = "--smallwg" in sys.argv  # one- and two-wave workgroups
NARROW_ONLY = "--narrow" in sys.argv  # 4- / 8- / 16-lane groups for short packets
PAIR_ONLY = "--pair" in sys.argv  # two packets a wave streamed as one run of chunks (k_ipv4_pair)
PASS_ONLY = "--pass" in sys.argv  # 6-KiB passes: a wave per packet (64 x 6), or 32 lanes x 12 loads

def equal_length(L, op):
    """Packets of L bytes each, as many as configs[3]'s bytes hold (uNNNN, uNNNN_rx)."""
    from tcp_amd.csum import PKT_DTYPE
    total = workload.make_batch("mixed").total_bytes
    n = total // L
    d = np.zeros(n, PKT_DTYPE)
    d["offset"] = np.arange(n, dtype=np.uint64) * np.uint64(L)
    d["len"] = L
    return workload.Batch("mixed", "ipv4", n, d, n * L, n * L, 0, op="rx" if op else "sums")


for cfg in ([a for a in sys.argv[1:] if not a.startswith("--")] or ["mixed", "mixed_aligned", "mixed_rx"]):
    b = equal_length(int(cfg[1:].split("_")[0]), cfg.endswith("_rx")) if cfg.startswith("u") else \
        workload.make_batch(cfg)
    arena, descs = workload.materialize(b)
    n = b.n
    rx = b.op == "rx"
    mode = 2 if rx else 0
    out0 = torch.empty(n, dtype=torch.uint32, device="cuda")
    v0 = torch.empty(n, dtype=torch.int8, device="cuda")
    if rx:
        tc.batch_ipv4_rx_verify(arena, descs, n, b.total_bytes, verdict=v0, out=out0, want_flags=False)
    else:
        tc.batch_ipv4(arena, descs, n, b.total_bytes, out=out0, want_flags=False)
    torch.cuda.synchronize()

    def product(o, v):
        if rx:
            tc.batch_ipv4_rx_verify(arena, descs, n, b.total_bytes, verdict=v, out=o, want_flags=False)
        else:
            tc.batch_ipv4(arena, descs, n, b.total_bytes, out=o, want_flags=False)

    def shape(wg, occ):
        def f(o, v):
            _lib.check(B.tcsum_probe_ipv4_shape(arena.data_ptr(), descs.data_ptr(), n, mode, wg, occ, o.data_ptr(),
                                                v.data_ptr(), torch.cuda.current_stream().cuda_stream),
                       "probe_ipv4_shape")
        return f

    kinds = {"product (256 threads)": product, "256 threads, same kernel (probe lib)": shape(256, 0)}

    def with_pf(f, pf):
        def g(o, v):
            with tc.debug(pf_dist=pf):
                f(o, v)
        return g

    if NARROW_ONLY:
        kinds = {"product (256 threads)": product}
        shapes = ((2, 4), (4, 2), (4, 3), (4, 4), (8, 3), (8, 4), (8, 6), (16, 3), (16, 4), (16, 6)) if rx else \
            ((2, 4), (2, 6), (4, 2), (4, 3), (4, 4), (4, 6), (8, 2), (8, 3), (8, 4), (8, 6), (8, 8), (16, 2), (16, 3),
             (16, 4), (16, 6))
        if "--tiny" in sys.argv:
            shapes = ((2, 4), (2, 6), (4, 2), (4, 3), (4, 4)) if not rx else ((2, 4), (4, 2), (4, 3), (4, 4))
        kinds.update({f"{g} lanes x {u}": shape(256, 1200 + 10 * g + u) if g < 16 else shape(256, 1360 + u)
                      for g, u in shapes})
        if not rx:
            kinds["32 lanes x 6"] = shape(256, 0)
    elif SMALLWG_ONLY:
        kinds.update({"64 threads (one wave)": shape(64, 0), "128 threads": shape(128, 0)})
    elif PAIR_ONLY:
        kinds.update({"pair stream, 64 x 6": shape(256, 1006), "pair stream, 64 x 4": shape(256, 1004)})
        if not rx:
            kinds["pair stream, 64 x 3"] = shape(256, 1003)
    elif PASS_ONLY:
        kinds.update({"64 lanes x 6 (a wave per packet)": shape(256, 964), "32 lanes x 12": shape(256, 932)})
    elif LDS_ONLY:
        if rx:
            def lanes32(o, v):
                with tc.debug(lanes=32, loads=6):
                    product(o, v)
            kinds.update({"LDS ring 16x6": shape(256, 800), "LDS ring 16x4": shape(256, 804),
                          "LDS ring 32x6": shape(256, 832), "product at 32 x 6 (no ring)": lanes32})
        else:
            kinds.update({"3rd header chunk as a dword (H1)": shape(256, 900), "LDS ring 32x6": shape(256, 800),
                          "LDS ring 32x6 + H1": shape(256, 905), "LDS ring 32x4": shape(256, 804),
                          "LDS ring 32x8": shape(256, 808), "LDS ring 16x6": shape(256, 816)})
    elif SDESC_ONLY:
        kinds.update({"descriptors by scalar loads": shape(256, 700)})
    elif HDRX_ONLY:
        kinds.update({"header from the data pass": shape(256, 600)})
    elif ROLL_ONLY:
        kinds.update({"rolling slots": shape(256, 500), "rolling, 4 loads": shape(256, 504),
                      "rolling, held to the route's waves/SIMD": shape(256, 506 if rx else 507)})
        if rx:
            kinds["rolling, 32 lanes x 6"] = shape(256, 532)
        else:
            kinds.update({"rolling, 8 loads": shape(256, 508), "rolling, 16 lanes x 6": shape(256, 516)})
    elif DYN_ONLY:
        kinds.update({f"dyn M={m}": shape(256, 300 + m) for m in ((2, 4, 8) if rx else (2, 4, 8, 16))})
        for w in ((6, 7) if rx else (7, 8)):  # M = 4 held to w waves per SIMD
            kinds[f"dyn M=4, {w} waves/SIMD"] = shape(256, 300 + 16 * w + 4)
    elif DB_ONLY:
        kinds.update({"two passes in flight": shape(256, 200),
                      "product, pf_dist 2048": with_pf(product, 2048),
                      "two passes in flight, pf_dist 2048": with_pf(shape(256, 200), 2048)})
    elif SKEW_ONLY:
        kinds.update({"data pass 16 B past the line": shape(256, 116)})
        if not rx:
            kinds["data pass 64 B past the line"] = shape(256, 164)
    elif rx:
        kinds.update({"1024 threads": shape(1024, 0), "<= 72 VGPRs (7 waves/SIMD)": shape(256, 7),
                      "<= 64 VGPRs (8 waves/SIMD)": shape(256, 8), "data pass 16 B past the line": shape(256, 116)})
    else:
        kinds.update({"512 threads": shape(512, 0), "1024 threads": shape(1024, 0),
                      "<= 64 VGPRs (8 waves/SIMD)": shape(256, 8), "data pass 16 B past the line": shape(256, 116),
                      "data pass 64 B past the line": shape(256, 164)})
    bufs = {k: (torch.empty(n, dtype=torch.uint32, device="cuda"), torch.empty(n, dtype=torch.int8, device="cuda"))
            for k in kinds}
    for k, fn in kinds.items():
        fn(*bufs[k])
        torch.cuda.synchronize()
        assert torch.equal(bufs[k][0], out0), k
        if rx:
            assert torch.equal(bufs[k][1], v0), k
    times = {k: [] for k in kinds}
    names = list(kinds)
    for r in range(7):
        for i in range(len(names)):  # the variant timed first rotates
            k = names[(r + i) % len(names)]
            fn = kinds[k]
            fn(*bufs[k])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                fn(*bufs[k])
            e1.record()
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / 10)
    alg = b.total_bytes + (17 if rx else 20) * n
    base = np.median(times["product (256 threads)"])
    print(f"# {cfg}: {n} packets, {b.total_bytes} B; median of 7 rounds x 10 launches, interleaved, first-timed rotated; results equal")
    for k, t in times.items():
        m = np.median(t)
        print(f"{k:42s} {m*1e3:9.1f} us  {m/base:6.3f}x  {alg / (m*1e-3) / 8e12:6.4f} of 8 TB/s", flush=True)
    del arena, descs, bufs
    torch.cuda.empty_cache()
