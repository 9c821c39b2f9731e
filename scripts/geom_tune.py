"""Geometry sweep (TCSUM_G x TCSUM_U) for one config, interleaved rounds,
median us per launch, results checked equal across geometries.
Usage: geom_tune.py CONFIG G:U,G:U,...  [XCD]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tcp_amd as tc  # noqa: E402
from tcp_amd import workload  # noqa: E402

cfg = sys.argv[1]
geoms = [tuple(int(v) for v in g.split(":")) for g in sys.argv[2].split(",")]
if len(sys.argv) > 3:
    os.environ["TCSUM_XCD"] = sys.argv[3]
rounds = 5
b = workload.make_batch(cfg)
arena, descs = workload.materialize(b)
out = torch.empty(b.n, dtype=torch.uint16 if b.kind == "peso" else torch.uint32, device="cuda")


verdict = torch.empty(b.n, dtype=torch.int8, device="cuda")
if cfg == "mixed_tx":  # fill once so every timed launch rewrites the same values
    tc.batch_ipv4_tx_fill(arena, descs, b.n, b.total_bytes, want_flags=False)


def run():
    if b.kind == "peso":
        tc.batch_peso(arena, descs, b.n, b.total_bytes, out=out)
    elif cfg == "mixed_tx":
        tc.batch_ipv4_tx_fill(arena, descs, b.n, b.total_bytes, out=out, want_flags=False)
    elif cfg == "mixed_rx":
        tc.batch_ipv4_rx_verify(arena, descs, b.n, b.total_bytes, verdict=verdict, out=out, want_flags=False)
    else:
        tc.batch_ipv4(arena, descs, b.n, b.total_bytes, out=out, want_flags=False)


times = {g: [] for g in geoms}
probe = []
ref = None
for r in range(rounds):
    for g in geoms:
        os.environ["TCSUM_G"], os.environ["TCSUM_U"] = str(g[0]), str(g[1])
        run()
        torch.cuda.synchronize()
        if ref is None:
            ref = out.clone()
        elif r == 0:
            assert torch.equal(ref, out), g
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            run()
        e1.record()
        torch.cuda.synchronize()
        times[g].append(e0.elapsed_time(e1) / 10)
    tc.probe_read(arena, b.arena_bytes)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        tc.probe_read(arena, b.arena_bytes)
    e1.record()
    torch.cuda.synchronize()
    probe.append(e0.elapsed_time(e1) / 10)
pus = np.median(probe) * 1e3
print(f"== {cfg} n={b.n} bytes={b.total_bytes} xcd={os.environ.get('TCSUM_XCD', 'default')}  "
      f"probe {pus:.1f} us {b.arena_bytes / pus / 1e3:.1f} GB/s", flush=True)
for g in geoms:
    us = np.median(times[g]) * 1e3
    print(f"  G={g[0]:2d} U={g[1]:2d}  {us:9.1f} us  {b.total_bytes / us / 1e3:8.1f} GB/s  "
          f"{pus / us:.3f} of probe  (min {min(times[g]) * 1e3:.1f})", flush=True)
