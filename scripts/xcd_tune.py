"""XCD-grouped block order (TCSUM_XCD = workgroups per XCD run) on every
bench workload: interleaved rounds in one process, median us per launch, and
results checked equal to the identity order."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tcp_amd as tc  # noqa: E402
from tcp_amd import workload  # noqa: E402

configs = sys.argv[1].split(",") if len(sys.argv) > 1 else ["mtu", "tso", "mixed", "mixed_tx", "mixed_rx"]
xgs = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [1, 2, 4, 8, 16, 32]
rounds = 5
for cfg in configs:
    b = workload.make_batch(cfg)
    arena, descs = workload.materialize(b)
    if cfg == "mixed_tx":  # fill once so every timed launch rewrites the same values
        tc.batch_ipv4_tx_fill(arena, descs, b.n, b.total_bytes, want_flags=False)
    out = torch.empty(b.n, dtype=torch.uint16 if b.kind == "peso" else torch.uint32, device="cuda")
    verdict = torch.empty(b.n, dtype=torch.int8, device="cuda")

    def run():
        if b.kind == "peso":
            tc.batch_peso(arena, descs, b.n, b.total_bytes, out=out)
        elif cfg == "mixed_tx":
            tc.batch_ipv4_tx_fill(arena, descs, b.n, b.total_bytes, out=out, want_flags=False)
        elif cfg == "mixed_rx":
            tc.batch_ipv4_rx_verify(arena, descs, b.n, b.total_bytes, verdict=verdict, out=out, want_flags=False)
        else:
            tc.batch_ipv4(arena, descs, b.n, b.total_bytes, out=out, want_flags=False)

    times = {x: [] for x in xgs}
    ref = None
    for r in range(rounds):
        for x in xgs:
            os.environ["TCSUM_XCD"] = str(x)
            run()
            torch.cuda.synchronize()
            if ref is None:
                ref = (out.clone(), verdict.clone())
            elif r == 0:
                assert torch.equal(ref[0], out) and torch.equal(ref[1], verdict), (cfg, x)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                run()
            e1.record()
            torch.cuda.synchronize()
            times[x].append(e0.elapsed_time(e1) / 10)
    print(f"== {cfg}: n={b.n} bytes={b.total_bytes}", flush=True)
    for x in xgs:
        us = np.median(times[x]) * 1e3
        print(f"  xcd={x:3d}  {us:9.1f} us  {b.total_bytes / us / 1e3:8.1f} GB/s  "
              f"(min {min(times[x]) * 1e3:.1f})", flush=True)
    # the read probe on the same bytes, same orders
    pt = {x: [] for x in xgs}
    for r in range(rounds):
        for x in xgs:
            os.environ["TCSUM_PROBE_XCD"] = str(x)
            tc.probe_read(arena, b.arena_bytes)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                tc.probe_read(arena, b.arena_bytes)
            e1.record()
            torch.cuda.synchronize()
            pt[x].append(e0.elapsed_time(e1) / 10)
    for x in xgs:
        us = np.median(pt[x]) * 1e3
        print(f"  probe xcd={x:3d}  {us:9.1f} us  {b.arena_bytes / us / 1e3:8.1f} GB/s", flush=True)
    del arena, descs, out
    torch.cuda.empty_cache()
