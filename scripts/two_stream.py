"""What do consecutive independent batches gain from overlapping launches?
configs[1] (1M x 1500-B packed segments, tcsum_batch_peso) launched R times
  1s   on one stream (the bench's step: each launch fills and drains the GPU)
  2s   alternating over two streams, each launch with its own out buffer
  4s   the same over four streams
The aggregate time of R launches is taken on the default stream after it
waits for every stream.  One process, interleaved rounds, first-timed leg
rotated; every leg's results checked equal to the one-stream leg's.

  python scripts/two_stream.py [ROUNDS]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tcp_amd as tc  # noqa: E402
from tcp_amd import workload  # noqa: E402

b = workload.make_batch("mtu")
arena, descs = workload.materialize(b)
n, nb = b.n, b.total_bytes
alg = nb + 26 * n
R = 20
main = torch.cuda.current_stream()
legs = {}
for ns in (1, 2, 4):
    streams = [main] if ns == 1 else [torch.cuda.Stream() for _ in range(ns)]
    outs = [torch.empty(n, dtype=torch.uint16, device="cuda") for _ in range(ns)]
    legs[f"{ns}s"] = (streams, outs)


def run(streams, outs):
    ev = torch.cuda.Event()
    ev.record(main)
    for s in streams:
        s.wait_event(ev)
    for i in range(R):
        k = i % len(streams)
        tc.batch_peso(arena, descs, n, nb, out=outs[k], stream=streams[k])
    for s in streams:
        if s is not main:
            main.wait_stream(s)


def timed(leg):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record(main)
    run(*leg)
    e1.record(main)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / R * 1e3


for leg in legs.values():
    run(*leg)
torch.cuda.synchronize()
ref = legs["1s"][1][0]
for k, (_, outs) in legs.items():
    for o in outs:
        assert torch.equal(o, ref), k
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 9
names = list(legs)
ts = {k: [] for k in names}
for r in range(rounds):
    for i in range(len(names)):
        k = names[(r + i) % len(names)]
        ts[k].append(timed(legs[k]))
print(f"# configs[1] {n} x 1500 B, {alg / 1e9:.4f} GB per launch; {rounds} rounds x {R} launches, "
      f"first-timed rotated; results equal", flush=True)
for k in names:
    us = float(np.median(ts[k]))
    print(f"{k:3s} {us:8.1f} us/launch  {alg / us / 1e3:8.1f} GB/s  frac {alg / us / 1e3 / 8000:.4f}  "
          f"(min {min(ts[k]):.1f} max {max(ts[k]):.1f})", flush=True)
