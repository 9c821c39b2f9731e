"""Launch-to-launch variance of the headline kernel (configs[1]: 1M x 1500 B
checksum_peso, k_segments_pk) -- VERDICT r05 item 5 (measurement script).

Per-launch HIP events on the launch stream around each tcsum_batch_peso,
in phases that isolate the suspects for the slow launches:

  b2b      N launches back to back (the bench's timed region)
  gap      launches each after an idle gap of GAP ms (clock / power ramp after idle)
  cpuload  back to back while 16 host processes spin (host-side interference)
  after_big  each launch right after a 16-GiB-read launch of another kernel
             (the bench's secondary configs / probes before and after)

Prints one JSON line per phase: mean / median / p90 / p99 / max in us,
mean over median, the indices of the launches above median * 1.02 and how
they fall (first of the phase, periodic, clustered), and a 64-bin
autocorrelation summary.  Run it under `rocprofv3 --kernel-trace` to get the
same launches' dispatch durations.

  python scripts/launch_variance.py [N]
"""
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tcp_amd as tc  # noqa: E402
from tcp_amd import workload  # noqa: E402


def summary(name, us, extra=None):
    us = np.asarray(us, dtype=np.float64)
    med = float(np.median(us))
    slow = np.nonzero(us > med * 1.02)[0]
    d = us - us.mean()
    ac = [float(np.dot(d[:-k], d[k:]) / max(1e-12, np.dot(d, d))) for k in range(1, min(65, us.size))]
    top = sorted(range(len(ac)), key=lambda k: -ac[k])[:3]
    line = {"phase": name, "launches": int(us.size), "mean_us": round(float(us.mean()), 2),
            "median_us": round(med, 2), "p90_us": round(float(np.percentile(us, 90)), 2),
            "p99_us": round(float(np.percentile(us, 99)), 2), "max_us": round(float(us.max()), 2),
            "min_us": round(float(us.min()), 2), "mean_over_median": round(float(us.mean()) / med, 4),
            "slow_count": int(slow.size), "slow_first_idx": [int(i) for i in slow[:20]],
            "slow_share_of_excess": round(float((us[slow] - med).sum() / max(1e-9, (us - med).clip(0).sum())), 3)
            if slow.size else 0.0,
            "first5_us": [round(float(x), 1) for x in us[:5]],
            "autocorr_top": [[k + 1, round(ac[k], 3)] for k in top]}
    if extra:
        line.update(extra)
    print(json.dumps(line), flush=True)
    return us


def _spin(stop):
    x = 0
    while not stop.is_set():
        for _ in range(100000):
            x += 1


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    b = workload.make_batch("mtu")
    arena, descs = workload.materialize(b)
    out = torch.empty(b.n, dtype=torch.uint16, device="cuda")
    big = torch.empty(16 << 30, dtype=torch.uint8, device="cuda")  # an HBM-sized other read
    sink = torch.zeros(1, dtype=torch.uint32, device="cuda")
    torch.cuda.synchronize()

    def one():
        tc.batch_peso(arena, descs, b.n, b.total_bytes, out=out)

    def timed(k, before=None, gap_ms=0.0):
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(k)]
        for a, e in evs:
            if before is not None:
                before()
            a.record()
            one()
            e.record()
            if gap_ms:
                torch.cuda.synchronize()
                time.sleep(gap_ms / 1e3)
        torch.cuda.synchronize()
        return [a.elapsed_time(e) * 1e3 for a, e in evs]

    for _ in range(20):  # warm
        one()
    torch.cuda.synchronize()
    b2b = summary("b2b", timed(n))
    # the same launches again, to see whether the b2b tail repeats at the same indices
    b2b2 = summary("b2b_again", timed(n))
    slow1 = set(np.nonzero(b2b > np.median(b2b) * 1.02)[0])
    slow2 = set(np.nonzero(b2b2 > np.median(b2b2) * 1.02)[0])
    print(json.dumps({"b2b_slow_indices_common": len(slow1 & slow2), "b2b_slow": len(slow1),
                      "b2b_again_slow": len(slow2)}), flush=True)
    summary("gap_2ms", timed(min(n, 300), gap_ms=2.0))
    summary("gap_20ms", timed(min(n, 100), gap_ms=20.0))

    ctx = mp.get_context("spawn")  # processes: spinning threads would hold this one's GIL
    stop = ctx.Event()
    procs = [ctx.Process(target=_spin, args=(stop,), daemon=True) for _ in range(16)]
    for p in procs:
        p.start()
    time.sleep(1.0)
    summary("cpuload_16procs", timed(n))
    stop.set()
    for p in procs:
        p.join(10)
    summary("after_16GiB_read", timed(min(n, 100), before=lambda: tc.probe_read(big, sink=sink)))
    # where in a long back-to-back run the slow launches sit: 10 blocks
    us = np.asarray(timed(4 * n))
    blocks = us.reshape(10, -1)
    print(json.dumps({"phase": "b2b_long_blocks", "launches": int(us.size),
                      "block_mean_us": [round(float(x), 2) for x in blocks.mean(1)],
                      "block_median_us": [round(float(np.median(x)), 2) for x in blocks],
                      "mean_over_median": round(float(us.mean() / np.median(us)), 4)}), flush=True)


if __name__ == "__main__":
    main()
