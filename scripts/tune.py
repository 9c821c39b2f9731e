"""Sweep kernel geometry (lanes per packet G, loads per lane U, nontemporal)
for each BASELINE config; interleaved rounds in one process (median ms)."""
import itertools
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tcp_amd as tc  # noqa: E402
from tcp_amd import workload  # noqa: E402

configs = sys.argv[1].split(",") if len(sys.argv) > 1 else ["mtu", "tso", "mixed"]
rounds = 3
for cfg in configs:
    b = workload.make_batch(cfg)
    arena, descs = workload.materialize(b)
    ref = None
    if b.kind == "peso":
        geoms = list(itertools.product((16, 32, 64), (1, 2, 3, 4, 6, 8, 16), (0, 1, 2)))
    else:
        geoms = list(itertools.product((16, 32, 64), (2, 4, 8, 16), (0,)))
    times = {g: [] for g in geoms}
    out = torch.empty(b.n, dtype=torch.uint16 if b.kind == "peso" else torch.uint32, device="cuda")
    for r in range(rounds):
        for g in geoms:
            os.environ["TCSUM_G"], os.environ["TCSUM_U"], os.environ["TCSUM_P"] = map(str, g)
            def run():
                if b.kind == "peso":
                    tc.batch_peso(arena, descs, b.n, b.total_bytes, out=out)
                else:
                    tc.batch_ipv4(arena, descs, b.n, b.total_bytes, out=out, want_flags=False)
            run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                run()
            e1.record()
            torch.cuda.synchronize()
            times[g].append(e0.elapsed_time(e1) / 10)
            if ref is None:
                ref = out.clone()
            elif r == 0:
                assert torch.equal(ref, out), g
    # achievable: plain streaming read of the same bytes, by loads per lane
    probe = {}
    for pu in (1, 2, 4, 8, 16):
        os.environ["TCSUM_PROBE_U"] = str(pu)
        ts = []
        for _ in range(rounds):
            tc.probe_read(arena, b.arena_bytes)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                tc.probe_read(arena, b.arena_bytes)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 10)
        probe[pu] = np.median(ts)
    del os.environ["TCSUM_PROBE_U"]
    alg = b.total_bytes + b.n * (26 if b.kind == "peso" else 20)
    rows = sorted((np.median(t), g) for g, t in times.items())
    print(f"== {cfg}: n={b.n} bytes={b.total_bytes}")
    for pu, ms in probe.items():
        print(f"  probe U={pu:2d}  {ms*1e3:8.1f} us  {b.arena_bytes/ms/1e6:7.1f} GB/s")
    for ms, g in rows[:25]:
        print(f"  G={g[0]:2d} U={g[1]:2d} P={g[2]}  {ms*1e3:8.1f} us  {alg/ms/1e6:7.1f} GB/s  {alg/ms/1e6/8000:.3f}")
    del arena, descs
    torch.cuda.empty_cache()
