"""A/B of route knobs (include/tcsum_debug.h, set per variant with
tcsum_debug_set; round 4 replaced the environment variables rounds 1-3 read)
in ONE process: interleaved rounds, median us per launch, and every
variant's results must equal the default's.

  python scripts/env_ab.py CONFIG KNOB=VALUE[,KNOB=VALUE...] ...
  e.g. python scripts/env_ab.py mixed_tx tx_split=0
  (the old names TCSUM_G / TCSUM_U / TCSUM_XCD / TCSUM_PACKED / TCSUM_TX_SPLIT
  are accepted and mapped to lanes / loads / xcd / packed / tx_split)
CONFIG: mtu | tso | mixed | mixed_tx | mixed_rx | mixed_txo
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tcp_amd as tc  # noqa: E402
from tcp_amd import workload  # noqa: E402

cfg = sys.argv[1]
variants = [{}] + [dict(kv.split("=", 1) for kv in a.split(",")) for a in sys.argv[2:]]
b = workload.make_batch(cfg)
arena, descs = workload.materialize(b)
n = b.n
peso = b.kind == "peso"
out = torch.empty(n, dtype=torch.uint16 if peso else torch.uint32, device="cuda")
verdict = torch.empty(n, dtype=torch.int8, device="cuda")
flags = torch.empty(n, dtype=torch.uint8, device="cuda")


def run():
    if peso:
        tc.batch_peso(arena, descs, n, b.total_bytes, out=out)
    elif b.op == "tx":
        tc.batch_ipv4_tx_fill(arena, descs, n, b.total_bytes, out=out, want_flags=False)
    elif b.op == "txo":
        tc.batch_ipv4_tx_offload(arena, descs, n, b.total_bytes, out=out, flags=flags)
    elif b.op == "rx":
        tc.batch_ipv4_rx_verify(arena, descs, n, b.total_bytes, verdict=verdict, out=out, want_flags=False)
    else:
        tc.batch_ipv4(arena, descs, n, b.total_bytes, out=out, want_flags=False)


OLD = {"TCSUM_G": "lanes", "TCSUM_U": "loads", "TCSUM_XCD": "xcd", "TCSUM_PACKED": "packed",
       "TCSUM_TX_SPLIT": "tx_split"}


def with_env(env, fn):
    knobs = {OLD.get(k, k): int(v) for k, v in env.items()}
    with tc.debug(**knobs):
        return fn()


# a tx fill writes the packets: every variant, run on the unfilled arena, must
# leave the same bytes as the default
arena_in = arena.clone() if b.op == "tx" else None
run()
torch.cuda.synchronize()
ref = (out.clone(), verdict.clone())
arena_ref = arena.clone() if b.op == "tx" else None
for v in variants[1:]:
    if arena_ref is not None:
        arena.copy_(arena_in)
    with_env(v, run)
    torch.cuda.synchronize()
    assert torch.equal(out, ref[0]) and torch.equal(verdict, ref[1]), f"{v} changed the results"
    if arena_ref is not None:
        assert torch.equal(arena, arena_ref), f"{v} changed the filled packets"
times = [[] for _ in variants]
for r in range(7):
    for j in range(len(variants)):  # the variant timed first rotates (it reads ~1 % slow)
        i = (r + j) % len(variants)
        v = variants[i]
        def timed():
            run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                run()
            e1.record()
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / 10
        times[i].append(with_env(v, timed))
base = np.median(times[0])
print(f"# {cfg}: {n} packets, {b.total_bytes} B; median of 7 rounds x 10 launches, interleaved, first-timed rotated")
for v, t in zip(variants, times):
    m = np.median(t)
    print(f"{(','.join(f'{k}={x}' for k, x in v.items()) or 'default'):40s} {m*1e3:9.1f} us  {m/base:6.3f}x")
