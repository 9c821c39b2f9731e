"""What a tx fill's scattered field writes cost by store granularity, on
configs[3]'s arena (1M mixed IPv4 packets, 64-9000 B, packed): the field
addresses the fill writes (tcsum_probe_txfloor_prepare), then the scatter
after a plain read of the bytes (so the fields' lines are not in cache),
writing each field as two byte stores (the product's k_tx_scatter form) or
as the whole 16 / 32 / 64 / 128 / 256-B aligned block holding it; beside the
read alone and the tx fill itself.  The fill, read and floor are timed first,
on the intact arena; the block variants junk it.  Interleaved rounds, median.

  python scripts/tx_scatter_gr_probe.py [ROUNDS]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tcp_amd as tc  # noqa: E402
from tcp_amd import workload  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 7
b = workload.make_batch("mixed_tx")
arena, descs = workload.materialize(b)
nbytes = arena.numel()
s = torch.cuda.current_stream()


def timed(fn, m=10):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(m):
        fn()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / m * 1e3  # us


def run(legs):
    names = list(legs)
    ts = {k: [] for k in names}
    for r in range(rounds):
        for i in range(len(names)):
            k = names[(r + i) % len(names)]
            ts[k].append(timed(legs[k]))
    return {k: sorted(v)[len(v) // 2] for k, v in ts.items()}


def fill_split(v, warm=None):
    with tc.debug(tx_split=v, tx_warm=warm):
        tc.batch_ipv4_tx_fill(arena, descs, b.n, b.total_bytes, want_flags=False)


def fill_warm(v):
    with tc.debug(tx_warm=v):
        tc.batch_ipv4_tx_fill(arena, descs, b.n, b.total_bytes, want_flags=False)


fh = tc.txfloor_prepare(arena, nbytes, descs, b.n, b.total_bytes)
# phase 1, on the intact arena: the fill, the read, the floor
res = run({
    "tx fill (route)": lambda: tc.batch_ipv4_tx_fill(arena, descs, b.n, b.total_bytes, want_flags=False),
    "tx fill in place (tx_split 0)": lambda: fill_split(0),
    "tx fill, cold scatter (tx_warm 0)": lambda: fill_warm(0),
    "read only": lambda: tc.probe_read(arena, nbytes),
    "floor: read + 2-B scatter": lambda: tc.probe_txfloor(fh, deferred=True),
    "floor: in-stream 2-B stores": lambda: tc.probe_txfloor(fh, deferred=False),
})
# phase 2 (junks the arena): the read, then the scatter by block size
legs = {f"read + {gr}-B block scatter": (lambda v=v: tc.probe_txfloor(fh, variant=v))
        for v, gr in zip(range(2, 8), (2, 16, 32, 64, 128, 256))}
legs["read + 64-B line RMW scatter"] = lambda: tc.probe_txfloor(fh, variant=8)
legs["read + atomic and/or scatter"] = lambda: tc.probe_txfloor(fh, variant=9)
legs["read + line load, then 2-B stores"] = lambda: tc.probe_txfloor(fh, variant=10)
legs["read + field dword load, then 2-B"] = lambda: tc.probe_txfloor(fh, variant=11)
legs["in-stream 64-B line writes"] = lambda: tc.probe_txfloor(fh, variant=12)
legs["in-stream, dword loaded, then 2-B"] = lambda: tc.probe_txfloor(fh, variant=13)
res.update(run(legs))
torch.cuda.synchronize()
pos = fh["fpos"].view(-1, 2)
have = (pos != -1)
print(f"# configs[3] arena {b.total_bytes} B, {b.n} packets, {int(have.sum())} fields; "
      f"median of {rounds} interleaved rounds x 10 launches", flush=True)
for k, v in res.items():
    print(f"{k:34s} {v:9.1f} us  {b.total_bytes / (v * 1e-6) / 8e12:7.4f} of 8 TB/s (batch bytes / time)", flush=True)
