"""Does holding waves back before their first load change the HBM stream rate?

tcsum_probe_segments (the headline kernel's own loads, no arithmetic) with
TCSUM_PROBE_PACE = k | flags: every wave sleeps k x s_sleep(1) (~64 cycles)
before its descriptor read; 0x100 staggers by wave in the workgroup, 0x200 by
workgroup.  Interleaved rounds with the product kernel, per-launch medians.

    python scripts/pace_probe.py [config] > gpurun_out/pace.txt
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import tcp_amd as tc  # noqa: E402
from tcp_amd import workload  # noqa: E402


def main():
    config = sys.argv[1] if len(sys.argv) > 1 else "mtu"
    torch.cuda.set_device(0)
    b = workload.make_batch(config)
    arena, descs = workload.materialize(b)
    out = torch.empty(b.n, dtype=torch.uint16, device="cuda")
    sink = torch.zeros(1, dtype=torch.uint32, device="cuda")
    alg = b.total_bytes + 26 * b.n
    paces = [0, 1, 2, 4, 8, 0x101, 0x102, 0x104, 0x201, 0x202, 0x204, 0x301]

    def probe(p):
        def f():
            os.environ["TCSUM_PROBE_PACE"] = str(p)
            tc.probe_segments(arena, descs, b.n, b.total_bytes, sink)
        return f

    kinds = {"product": lambda: tc.batch_peso(arena, descs, b.n, b.total_bytes, out=out)}
    for p in paces:
        kinds[f"pace_{p:#x}"] = probe(p)
    for fn in kinds.values():  # warm
        for _ in range(5):
            fn()
    torch.cuda.synchronize()
    per = {k: [] for k in kinds}
    m = 10
    s = torch.cuda.current_stream()
    for _ in range(7):
        for k, fn in kinds.items():
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(m):
                fn()
            e1.record(s)
            torch.cuda.synchronize()
            per[k].append(e0.elapsed_time(e1) / m)
    print(f"config {config}: {b.n} segments, algorithmic {alg} B; per-launch median over 7 rounds x {m}")
    for k, v in per.items():
        med = sorted(v)[len(v) // 2]
        print(f"{k:>12}  {med * 1e3:8.1f} us  {alg / (med * 1e-3) / 1e9:7.1f} GB/s  "
              f"spread {min(v) * 1e3:.1f}-{max(v) * 1e3:.1f}")
    assert int(sink.item()) == 0


if __name__ == "__main__":
    main()
