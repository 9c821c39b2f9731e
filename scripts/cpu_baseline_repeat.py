"""The all-core CPU baseline, repeated: the bench's own
cpu_baseline sample for configs[1], [2] and [3] (the first >= 1 GiB of the
batch; for IPv4 packets their L4 ranges), timed by the reference's
checksum_peso on every logical CPU R times in one process, each timing thread
pinned and first-touching its slice (oracle/csum_oracle.c orc_time_peso).

  python scripts/cpu_baseline_repeat.py [repeats] [seconds]
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import tcp_amd as tc  # noqa: E402
from oracle import pyoracle  # noqa: E402
from tcp_amd import workload  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
secs = float(sys.argv[2]) if len(sys.argv) > 2 else 4.0
pyoracle.build()
threads = min(256, os.cpu_count() or 1)
res = {"host_cpu": bench.cpu_model(), "threads": threads, "seconds_per_run": secs, "configs": {}}
for cfg in ("mtu", "tso", "mixed"):
    b = workload.make_batch(cfg)
    arena, descs = workload.materialize(b)
    out = torch.empty(b.n, dtype=torch.uint16 if b.kind == "peso" else torch.uint32, device="cuda")
    if b.kind == "peso":
        tc.batch_peso(arena, descs, b.n, b.total_bytes, out=out)
    else:
        tc.batch_ipv4(arena, descs, b.n, b.total_bytes, out=out, want_flags=False)
    torch.cuda.synchronize()
    r = {"batch": b, "arena": arena, "out": out}
    lens = b.descs["len"].astype(np.int64)
    n = max(1, min(b.n, int(np.searchsorted(np.cumsum(lens), min(b.total_bytes, 1 << 30))) + 1))
    end = int(b.descs["offset"][n - 1] + b.descs["len"][n - 1])
    host = arena[: end + 16].cpu().numpy()
    if b.kind == "peso":
        segs = b.descs[:n].copy()
    else:
        off = b.descs["offset"][:n].astype(np.int64)
        hdr = host[off[:, None] + np.arange(20)[None, :]]
        segs = np.zeros(n, pyoracle.PESO_DTYPE)
        segs["offset"], segs["len"] = off + 20, b.descs["len"][:n] - 20
        segs["src"], segs["dst"], segs["protocol"] = hdr[:, 12:16], hdr[:, 16:20], hdr[:, 9]
    runs = []
    for _ in range(reps):
        rate, _, _ = pyoracle.time_peso(host, segs, threads, secs, kind="reference")
        runs.append(round(rate / bench.GIB, 2))
    one, _, _ = pyoracle.time_peso(host, segs, 1, secs, kind="reference")
    res["configs"][cfg] = {"sample_bytes": int(segs["len"].sum()), "value_all_runs": runs,
                           "spread_max_over_min": round(max(runs) / min(runs), 3),
                           "value_1_thread": round(one / bench.GIB, 2)}
    print(cfg, res["configs"][cfg], flush=True)
    del arena, descs, out, host, r
    torch.cuda.empty_cache()
print(json.dumps(res))
