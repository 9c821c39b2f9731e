"""What separates the byte-window stream's load phase from the TSO kernel's
on configs[3]'s arena (one process, interleaved rounds, median us per
launch): the same W-wave windows read with nothing before the loads, behind
one or two shared scalar loads (k_flat_ipv4's plan), behind a descriptor of
their own (k_segments_wgx's), beside the TSO kernel itself over the arena cut
into 64-KiB ranges (product and its load probe), k_ipv4 and the flat probe's
loads-only form (tcsum_probe_window / tcsum_probe_flat, libtcsum_bench.so).

  python scripts/window_probe.py
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tcp_amd as tc  # noqa: E402
from tcp_amd import _lib, workload  # noqa: E402
from tcp_amd.csum import PESO_DTYPE  # noqa: E402

B = _lib.bench_lib()
b = workload.make_batch("mixed")
arena, descs = workload.materialize(b)
n = b.n
nbytes = b.arena_bytes
out = torch.empty(n, dtype=torch.uint32, device="cuda")
sink = torch.zeros(1, dtype=torch.uint32, device="cuda")
word = torch.zeros(4, dtype=torch.int64, device="cuda")
L64 = 65536
n64 = nbytes // L64
p64 = np.zeros(n64, PESO_DTYPE)
p64["offset"] = np.arange(n64, dtype=np.uint64) * np.uint64(L64)
p64["len"] = L64
p64["protocol"] = 6
d64 = tc.descs_to_device(p64)
o64 = torch.empty(n64, dtype=torch.uint16, device="cuda")
# one 24-B descriptor per workgroup for dep 3 (the smallest window: 4x3 = 12 KiB)
nd = nbytes // (16 * 64 * 4 * 3) + 2
dws = torch.zeros(nd * 24, dtype=torch.uint8, device="cuda")
s = lambda: torch.cuda.current_stream().cuda_stream


def window(w, u, dep):
    def f():
        _lib.check(B.tcsum_probe_window(arena.data_ptr(), nbytes, w, u, dep, word.data_ptr(), dws.data_ptr(), nd,
                                        sink.data_ptr(), s()), "probe_window")
    return f


def flat_v1(w, u):
    def f():
        _lib.check(B.tcsum_probe_flat(arena.data_ptr(), descs.data_ptr(), n, b.total_bytes, 1, w, u, sink.data_ptr(),
                                      1, None, s()), "probe_flat")
    return f


kinds = {"k_ipv4 (product)": lambda: tc.batch_ipv4(arena, descs, n, b.total_bytes, out=out, want_flags=False),
         "64-KiB ranges, k_segments_wgx (product)": lambda: tc.batch_peso(arena, d64, n64, n64 * L64, out=o64),
         "64-KiB ranges, its load probe": lambda: tc.probe_segments(arena, d64, n64, n64 * L64, sink),
         "plain read probe": lambda: tc.probe_read(arena, nbytes, sink),
         "flat 16x4 v1 (plan pass + loads)": flat_v1(16, 4)}
NAMES = {0: "nothing first", 1: "1 shared scalar word first", 2: "2 dependent shared words first",
         3: "own descriptor first", 4: "shifted 16 B", 5: "+ default-policy edge chunks",
         6: "shifted 16 B + edge chunks", 7: "shifted + edges + own descriptor (wgx's pattern)"}
for w, u, deps in ((16, 4, range(8)), (8, 4, (0, 4, 6)), (4, 3, (0, 4, 6))):
    for dep in deps:
        kinds[f"window {w}x{u}: {NAMES[dep]}"] = window(w, u, dep)
times = {k: [] for k in kinds}
for k, fn in kinds.items():
    fn()
torch.cuda.synchronize()
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
base = np.median(times["k_ipv4 (product)"])
print(f"# mixed arena: {nbytes} B; median of 7 rounds x 10 launches, interleaved; of 8 TB/s on the arena's bytes")
for k, t in times.items():
    m = np.median(t)
    print(f"{k:62s} {m*1e3:9.1f} us  {m/base:6.3f}x  {nbytes / (m*1e-3) / 8e12:6.4f}", flush=True)
