"""Capture-file rx verify, end to end: a 1M-frame raw-IPv4 savefile of
configs[3]-style packets (64-9000 B, tx-filled by the stack's rules) in pinned
host memory -> tcsum_pcap_index (host) -> tcsum_host_batch_ipv4_rx_verify over
the file in place; and the same file resident in HBM through
tcsum_batch_ipv4_rx_verify.  Measurement script, not product code."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tcp_amd as tc  # noqa: E402
from tcp_amd import pcap, workload  # noqa: E402

GIB = 1 << 30
n = int(os.environ.get("PCAP_FRAMES", 1 << 20))
b = workload.make_batch("mixed_rx", n=n)
lens = b.descs["len"].astype(np.uint64)
NG = os.environ.get("PCAP_NG") == "1"  # pcapng: SHB + IDB, then one Enhanced Packet Block per frame
if NG:
    blen = np.uint64(32) + (lens + np.uint64(3)) // np.uint64(4) * np.uint64(4)
    head, data_at = 48, 28
else:
    blen = lens + np.uint64(16)
    head, data_at = 24, 16
rec = np.zeros(n, np.uint64)
np.cumsum(blen[:-1], out=rec[1:])
rec += np.uint64(head)
file_bytes = int(rec[-1] + blen[-1])
descs = np.zeros(n, tc.PKT_DTYPE)
descs["offset"] = rec + np.uint64(data_at)
descs["len"] = lens

# packets generated in HBM where the capture holds them, filled like a sender
dev = torch.empty(file_bytes + 64, dtype=torch.uint8, device="cuda")
tc.synth_fill(dev, file_bytes + 64, 0, b.seed)
d_descs = tc.descs_to_device(descs)
tc.synth_ipv4(dev, d_descs, n, b.seed)
tc.batch_ipv4_tx_fill(dev, d_descs, n, int(lens.sum()), want_flags=False)
torch.cuda.synchronize()
host = tc.HostArena(file_bytes)
host.array[:] = dev[:file_bytes].cpu().numpy()
# savefile header (LINKTYPE_RAW) and record headers, written around the packets
if NG:
    host.array[:48] = np.frombuffer(np.array([0x0A0D0D0A, 28, 0x1A2B3C4D, 1, 0xFFFFFFFF, 0xFFFFFFFF, 28,
                                              1, 20, 101, 262144, 20], "<u4").tobytes(), np.uint8)
    hdr = np.zeros((n, 7), "<u4")
    hdr[:, 0] = 6
    hdr[:, 1] = blen
    hdr[:, 4] = np.arange(n)
    hdr[:, 5] = lens
    hdr[:, 6] = lens
    idx = rec[:, None].astype(np.int64) + np.arange(28)
    host.array[idx] = hdr.view(np.uint8).reshape(n, 28)
    tail = (rec + blen - np.uint64(4))[:, None].astype(np.int64) + np.arange(4)
    host.array[tail] = blen.astype("<u4").view(np.uint8).reshape(n, 4)
else:
    host.array[:24] = np.frombuffer(np.array([0xA1B2C3D4, 0x00040002, 0, 0, 262144, 101], "<u4").tobytes(),
                                    np.uint8)
    hdr = np.zeros((n, 4), "<u4")
    hdr[:, 0] = np.arange(n)
    hdr[:, 2] = lens
    hdr[:, 3] = lens
    idx = rec[:, None].astype(np.int64) + np.arange(16)
    host.array[idx] = hdr.view(np.uint8).reshape(n, 16)
dev[:file_bytes].copy_(torch.from_numpy(host.array[:file_bytes]))
total = int(lens.sum())
print(f"{'pcapng' if NG else 'classic'} capture: {n} frames, {file_bytes / GIB:.2f} GiB file, "
      f"{total / GIB:.2f} GiB of IPv4", flush=True)

buf = host.array[:file_bytes]
t = []
for _ in range(5):
    t0 = time.perf_counter()
    pk, l2 = pcap.index(buf)
    t.append(time.perf_counter() - t0)
assert (pk["offset"] == descs["offset"]).all() and (pk["len"] == descs["len"]).all() and (l2 == 0).all()
ti = float(np.median(t))
print(f"tcsum_pcap_index (16 thr x 4 chains) {ti * 1e3:8.2f} ms   {n / ti / 1e6:7.1f} Mframes/s", flush=True)

v, _, _, _ = pcap.rx_verify(buf)  # warm (staging, contexts)
t = []
for _ in range(3):
    t0 = time.perf_counter()
    v, l2, out, flags = pcap.rx_verify(buf)
    t.append(time.perf_counter() - t0)
tv = float(np.median(t))
assert (v == 0).all(), np.unique(v, return_counts=True)
print(f"pcap.rx_verify pinned file in place    {tv * 1e3:8.2f} ms   {total / tv / GIB:7.2f} GiB/s (index incl.)",
      flush=True)

t = []
for _ in range(3):
    t0 = time.perf_counter()
    tc.host_batch_ipv4_rx_verify(buf, pk)
    t.append(time.perf_counter() - t0)
tv = float(np.median(t))
print(f"  of which host_batch_ipv4_rx_verify   {tv * 1e3:8.2f} ms   {total / tv / GIB:7.2f} GiB/s", flush=True)

d_pk = tc.descs_to_device(pk)
verdict, _ = tc.batch_ipv4_rx_verify(dev, d_pk, n, total)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for _ in range(50):  # clocks up (bench.py's settle)
    tc.batch_ipv4_rx_verify(dev, d_pk, n, total, verdict=verdict)
s.record()
for _ in range(20):
    tc.batch_ipv4_rx_verify(dev, d_pk, n, total, verdict=verdict)
e.record()
e.synchronize()
ms = [s.elapsed_time(e) / 20]
assert int((verdict != 0).sum().item()) == 0
md = float(np.median(ms))
print(f"rx verify, file resident in HBM        {md:8.3f} ms   {total / (md * 1e-3) / GIB:7.1f} GiB/s", flush=True)
host.free()
