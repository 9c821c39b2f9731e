#!/usr/bin/env python3
"""Benchmark: Internet-checksum GiB/s, device-resident, on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]

One "step" = one batched checksum pass (one kernel launch) over the whole
synthetic batch already resident in HBM.  Before the K timed steps: W untimed
warm-up steps, continued (untimed) until --settle-ms have passed, so the GPU
clocks are out of idle whatever W the caller picks.  The headline workload is
BASELINE.json configs[1]: 1,048,576 x 1500 B TCP segments per GPU, checksummed
exactly as checksum_peso (net/src/tools.c:56-75) does, pseudo-header built
in-kernel.  With N GPUs every rank holds its own 1M-segment slice of one
N x 1M batch (configs[4] at N=8): weak scaling, no collective on the data path.

At N=1 the same JSON line also carries
  * configs[2] (256K x 64 KiB) and configs[3] (1M mixed IPv4, 64-9000 B),
  * roofline: algorithmic bytes / kernel time vs the 8 TB/s HBM3E peak, and
    the rocprofv3 PMC traffic (FETCH_SIZE x 2 + WRITE_SIZE, gfx950 correction),
  * cpu_baseline: the REFERENCE's own checksum_peso (oracle/_ref, compiled from
    the reference sources) on the host cores, on a bounded sample,
  * e2e: pinned host arena -> H2D -> kernel -> D2H.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GIB = float(1 << 30)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip table)
METRIC = "Internet-checksum GiB/s (device-resident), 1500B & 64KB packet batches"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=50,
                    help="untimed launches first: ~10 ms of load brings the GPU out of its idle clocks "
                         "(scripts/drift_probe.py: the first ~40 configs[1] launches run 6 %% slower)")
    ap.add_argument("--config", default="mtu", help="headline workload (mtu|tso|mixed|mixed_aligned)")
    ap.add_argument("--secondary", default="tso,mixed,mixed_aligned,mixed_tx,mixed_txo,mixed_rx",
                    help="extra configs measured at N=1")
    ap.add_argument("--settle-ms", type=float, default=30.0,
                    help="untimed: the warm-up also lasts at least this long (GPU clocks out of idle "
                         "whatever W is; 0 = exactly W launches)")
    ap.add_argument("--no-pmc", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args()


def algorithmic_bytes(batch) -> int:
    """Bytes one launch must move: every packet byte once, its descriptor, its result.

    peso: 24-B descriptor + 2-B result; ipv4 sums: 16-B descriptor + 4-B result;
    tx fill: 16 B + 4 B written into the packet; rx verify: 16 B + 1-B verdict;
    tx offload: 16 B + 4-B value + 1-B flags."""
    if batch.kind == "peso":
        per = 24 + 2
    else:
        per = {"sums": 16 + 4, "tx": 16 + 4, "rx": 16 + 1, "txo": 16 + 4 + 1}[batch.op]
    return batch.total_bytes + per * batch.n


def launch(tc, batch, arena, descs, out, flags=None):
    if batch.kind == "peso":
        tc.batch_peso(arena, descs, batch.n, batch.total_bytes, out=out)
    elif batch.op == "tx":
        tc.batch_ipv4_tx_fill(arena, descs, batch.n, batch.total_bytes, want_flags=False)
    elif batch.op == "txo":
        tc.batch_ipv4_tx_offload(arena, descs, batch.n, batch.total_bytes, out=out, flags=flags)
    elif batch.op == "rx":
        tc.batch_ipv4_rx_verify(arena, descs, batch.n, batch.total_bytes, verdict=out, want_flags=False)
    else:
        tc.batch_ipv4(arena, descs, batch.n, batch.total_bytes, out=out, want_flags=False)


SETTLE_MS = 30.0  # set from --settle-ms in main()


def time_config(torch, tc, workload, config, rank, steps, warmup, dist=None):
    batch = workload.make_batch(config, rank=rank)
    arena, descs = workload.materialize(batch)
    dt = torch.uint16 if batch.kind == "peso" else torch.int8 if batch.op == "rx" else torch.uint32
    out = torch.empty(batch.n, dtype=dt, device=arena.device)
    flags = torch.empty(batch.n, dtype=torch.uint8, device=arena.device) if batch.op == "txo" else None
    for _ in range(warmup):
        launch(tc, batch, arena, descs, out, flags)
    torch.cuda.synchronize()
    # untimed: keep warming until SETTLE_MS have passed (after idle the first
    # ~13 ms of launches run ~6 % slow while the clocks ramp,
    # profiles/r01/drift_probe.txt), so a small W does not time the ramp
    settle0 = time.perf_counter()
    while (time.perf_counter() - settle0) * 1e3 < SETTLE_MS:
        for _ in range(4):
            launch(tc, batch, arena, descs, out, flags)
        torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    wall0 = time.perf_counter()
    t0.record(stream)
    for _ in range(steps):
        launch(tc, batch, arena, descs, out, flags)
    t1.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - wall0
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    ms = t0.elapsed_time(t1)  # events on the launch stream: pure kernel time of K launches
    # the achievable side: a plain streaming read of the same bytes, same loads
    sink = torch.zeros(1, dtype=torch.uint32, device=arena.device)
    for _ in range(2):
        tc.probe_read(arena, batch.arena_bytes, sink)
    p0 = torch.cuda.Event(enable_timing=True)
    p1 = torch.cuda.Event(enable_timing=True)
    p0.record(stream)
    for _ in range(steps):
        tc.probe_read(arena, batch.arena_bytes, sink)
    p1.record(stream)
    torch.cuda.synchronize()
    probe_gbs = batch.arena_bytes / (p0.elapsed_time(p1) / steps * 1e-3) / 1e9
    return dict(batch=batch, arena=arena, descs=descs, out=out, ms=ms, wall_s=wall, probe_gbs=probe_gbs)


def result_entry(r, steps):
    b = r["batch"]
    ms_step = r["ms"] / steps
    alg = algorithmic_bytes(b)
    ach = alg / (ms_step * 1e-3) / 1e9
    return {
        "workload": b.config,
        "packets": b.n,
        "payload_bytes": b.total_bytes,
        "gib_s": b.total_bytes / (ms_step * 1e-3) / GIB,
        "ms_per_step": ms_step,
        "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(ach / HBM_PEAK_GBS, 4),
                     "achievable_read": round(r["probe_gbs"], 1),
                     "frac_of_achievable": round(ach / r["probe_gbs"], 4)},
    }


# ------------------------------------------------------------ PMC traffic

def pmc_traffic(config: str):
    """HBM bytes per launch from rocprofv3 counters, in separate passes
    (FETCH_SIZE, then WRITE_SIZE), run as a child before this process touches
    the GPU.  gfx950: FETCH_SIZE counts half the bytes of a wide streaming read
    (MI355X_MICROARCH.md §HBM) -> x2; both counters are in KiB."""
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None, "rocprofv3 not found"
    vals = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix=f"tcsum_pmc_{counter}_")
        cmd = [prof, "--pmc", counter, "--output-format", "csv", "-d", d, "-o", "pmc", "--",
               sys.executable, os.path.abspath(__file__), "--pmc-child", "--config", config,
               "--steps", "3", "--warmup", "1"]
        try:
            subprocess.run(cmd, check=True, timeout=240, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                           env=dict(os.environ, TMPDIR=d))
        except (subprocess.SubprocessError, OSError) as e:
            return None, f"rocprofv3 {counter} pass failed: {type(e).__name__}"
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        keep = os.environ.get("TCSUM_PMC_KEEP")  # directory to keep the raw counter CSVs in
        if keep:
            os.makedirs(keep, exist_ok=True)
            for i, f in enumerate(files):
                shutil.copy(f, os.path.join(keep, f"pmc_{counter.lower()}_{config}{'_%d' % i if i else ''}.csv"))
        per = []
        for f in files:
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    name = row.get("Kernel_Name", "")
                    if "k_segments" in name or "k_ipv4" in name:  # the checksum kernels only
                        if row.get("Counter_Name", counter) == counter:
                            per.append(float(row["Counter_Value"]))
        shutil.rmtree(d, ignore_errors=True)
        if not per:
            return None, f"no {counter} rows for the checksum kernel"
        vals[counter] = sorted(per)[len(per) // 2]
    traffic = vals["FETCH_SIZE"] * 1024 * 2 + vals["WRITE_SIZE"] * 1024
    return traffic, None


# ------------------------------------------------------------ CPU baseline

def cpu_model():
    """The GPU box's host CPU as /proc/cpuinfo names it (and its logical CPUs)."""
    try:
        with open("/proc/cpuinfo") as f:
            names = [ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")]
        return f"{names[0]} ({len(names)} logical CPUs on the host)" if names else None
    except OSError:
        return None


def cpu_baseline(torch, r, seconds):
    """The reference's checksum_peso (oracle/_ref/libtcpref.so, compiled from
    /root/reference; else the oracle port) on a bounded sample of the same
    segments, on this host's cores."""
    from oracle import pyoracle
    import numpy as np
    pyoracle.build()
    b = r["batch"]
    n = min(b.n, 65536 if b.config == "mtu" else 2048 if b.kind == "peso" else 16384)
    end = int(b.descs["offset"][n - 1] + b.descs["len"][n - 1])
    host = r["arena"][: end + 16].cpu().numpy()
    what = "segments"
    if b.kind == "peso":
        segs = b.descs[:n].copy()
        want = int(r["out"][:n].to(torch.int64).sum().item())
    else:
        # IPv4 packets: the reference's per-packet cost is checksum_peso over
        # the L4 bytes (tcp_in.c:80 / udp.c:410) plus checksum16 over the
        # 20-byte header (ipv4.c:243, ~0.5 % of the bytes, not timed); the
        # synthetic packets are IHL 5 with total_len == frame length
        off = b.descs["offset"][:n].astype(np.int64)
        hdr = host[off[:, None] + np.arange(20)[None, :]]
        segs = np.zeros(n, pyoracle.PESO_DTYPE)
        segs["offset"] = off + 20
        segs["len"] = b.descs["len"][:n] - 20
        segs["src"] = hdr[:, 12:16]
        segs["dst"] = hdr[:, 16:20]
        segs["protocol"] = hdr[:, 9]
        want = int((r["out"][:n].to(torch.int64) >> 16).sum().item())
        what = "packets' L4 ranges"
    rate1, kind, cs1 = pyoracle.time_peso(host, segs, 1, seconds, use_reference=True)
    threads = min(16, os.cpu_count() or 1)
    rateN, _, csN = pyoracle.time_peso(host, segs, threads, seconds / 2, use_reference=True)
    return {
        "value": round(rate1 / GIB, 3), "unit": "GiB/s", "cores": 1, "kind": kind,
        "sample": f"first {n} {what} of the {b.config} batch ({int(segs['len'].sum()) / 1e6:.0f} MB), "
                  f"re-summed for >= {seconds:.0f} s",
        "multi": {"value": round(rateN / GIB, 3), "cores": threads},
        "host_cpu": cpu_model(),
        "parity": bool(cs1 == want and csN == want),
    }


# ------------------------------------------------------------ end to end

def e2e(torch, tc, r):
    """tcsum_host_batch_peso from a pinned host arena (PCIe-inclusive)."""
    import ctypes
    import numpy as np
    from tcp_amd import _lib
    b = r["batch"]
    if b.kind != "peso":
        return None
    L = _lib.lib()
    nbytes = b.alloc_bytes
    p = L.tcsum_host_alloc(nbytes)
    if not p:
        return None
    try:
        host = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p))
        host[:] = r["arena"][:nbytes].cpu().numpy()
        out = np.zeros(b.n, np.uint16)
        tc.host_batch_peso(host, b.descs)  # warm (allocates device buffers)
        t0 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            out = tc.host_batch_peso(host, b.descs)
        dt = (time.perf_counter() - t0) / reps
        same = bool((out == r["out"].cpu().numpy()).all())
        # the host link itself: one plain pinned -> device copy of the same bytes
        src = torch.from_numpy(host)
        dst = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        link = nbytes / ((time.perf_counter() - t0) / reps) / GIB
        del dst
        res = {"gib_s": round(b.total_bytes / dt / GIB, 2), "ms_per_batch": round(dt * 1e3, 3),
               "path": "pinned host -> hipMemcpyAsync H2D (>= 64 MiB chunks in order on one copy stream, kernels on a second stream behind per-chunk events) -> kernel -> D2H",
               "h2d_copy_gib_s": round(link, 2),
               "matches_device_resident": same}
        ndev = torch.cuda.device_count()
        if ndev > 1:  # the same host batch sharded over every GPU of the node
            devs = list(range(ndev))
            out = tc.host_batch_peso_multi(host, b.descs, devs)
            t0 = time.perf_counter()
            for _ in range(reps):
                out = tc.host_batch_peso_multi(host, b.descs, devs)
            dt = (time.perf_counter() - t0) / reps
            res["multi_device"] = {"gpus": ndev, "gib_s": round(b.total_bytes / dt / GIB, 2),
                                   "matches_device_resident": bool((out == r["out"].cpu().numpy()).all())}
        return res
    finally:
        L.tcsum_host_free(p)


def legacy_latency(tc):
    """Per-call wall time of the synchronous drop-in symbols, the way the
    stack calls them per packet: checksum16 on a 20-B IPv4 header (ipv4.c:243)
    and checksum_peso on a 1500-B segment in 127-B blocks (tcp_out.c:20)."""
    import numpy as np
    hdr = bytes.fromhex("450000730000400040110000c0a80001c0a800c7")
    seg = np.random.default_rng(1).integers(0, 256, 1500, dtype=np.uint8).tobytes()
    buf = tc.PktBuf([seg[i: i + 127] for i in range(0, 1500, 127)])
    d, s_ = tc.IpAddr.v4([192, 168, 74, 3]), tc.IpAddr.v4([192, 168, 74, 2])
    res = {}
    for served in (False, True):  # one launch + sync per call / the call server's resident wave
        if served:
            tc.call_server(True)
        try:
            for name, fn in (("checksum16_20B_us", lambda: tc.checksum16(0, hdr, 20, 0, 1)),
                             ("checksum_peso_1500B_us", lambda: tc.checksum_peso(buf, d, s_, 6))):
                for _ in range(20):
                    fn()
                t0 = time.perf_counter()
                reps = 2000
                for _ in range(reps):
                    fn()
                res[("served_" if served else "") + name] = round((time.perf_counter() - t0) / reps * 1e6, 2)
        finally:
            if served:
                tc.call_server(False)
    res["note"] = ("plain: one launch + one sync per call; served_: tcsum_call_server (one resident wave "
                   "polling pinned memory). Use the batch API for throughput")
    return res


def main():
    args = parse()
    from tcp_amd import dist as D
    rank, local, world = D.env()
    n_gpus = max(world, 1)

    traffic, pmc_note = None, "skipped"
    if not args.pmc_child and world == 1 and not args.no_pmc:
        traffic, pmc_note = pmc_traffic(args.config)  # before this process touches the GPU

    import torch
    from tcp_amd import build
    build.build()
    import tcp_amd as tc
    from tcp_amd import workload

    # one process per GPU; TCSUM_DIST_BACKEND=gloo rehearses N ranks on fewer
    # GPUs (ranks share devices round-robin; RCCL refuses two ranks per GPU)
    backend = os.environ.get("TCSUM_DIST_BACKEND", "nccl")
    dev = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    dist = D.init(backend, dev)  # barrier + max-time only; no data-path collective

    global SETTLE_MS
    SETTLE_MS = 0.0 if args.pmc_child else max(0.0, args.settle_ms)
    if args.pmc_child:
        time_config(torch, tc, workload, args.config, 0, args.steps, args.warmup)
        return

    head = time_config(torch, tc, workload, args.config, rank, args.steps, args.warmup, dist)
    ms = D.max_over_ranks(dist, head["ms"], device="cuda" if backend == "nccl" else "cpu")
    b = head["batch"]
    ms_step = ms / args.steps
    value = n_gpus * b.total_bytes * args.steps / (ms * 1e-3) / GIB
    entry = result_entry(dict(head, ms=ms), args.steps)
    roof = dict(entry["roofline"])
    roof["traffic"] = (round(traffic) if traffic is not None else None)
    if traffic is None:
        roof["traffic_note"] = pmc_note
    else:
        roof["traffic_vs_algorithmic"] = round(traffic / algorithmic_bytes(b), 4)

    line = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "settle_ms": SETTLE_MS,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u16",
        "data": "synthetic: splitmix64 bytes generated in HBM, random src/dst (seed 20240807)",
        "config": {"workload": workload.CONFIG_NAMES[args.config], "packets_per_gpu": b.n,
                   "payload_bytes_per_gpu": b.total_bytes, "routine": "checksum_peso (tools.c:56-75)"
                   if b.kind == "peso" else "IPv4 header + L4 (ipv4.c:243, tcp_in.c:80, udp.c:410)",
                   "parallelism": f"{n_gpus} independent GPU shards, no collective"},
        "roofline": roof,
    }

    if world == 1:
        if not args.no_cpu:
            try:
                line["cpu_baseline"] = cpu_baseline(torch, head, args.cpu_seconds)
            except Exception as e:  # reported, never fatal to the GPU numbers
                line["cpu_baseline"] = {"value": None, "error": repr(e)}
        if not args.no_e2e:
            try:
                line["e2e"] = e2e(torch, tc, head)
            except Exception as e:
                line["e2e"] = {"error": repr(e)}
            try:
                line["legacy_sync_call"] = legacy_latency(tc)
            except Exception as e:
                line["legacy_sync_call"] = {"error": repr(e)}
        del head
        torch.cuda.empty_cache()
        extra = {}
        for cfg in [c for c in args.secondary.split(",") if c and c != args.config]:
            r = time_config(torch, tc, workload, cfg, 0, max(5, args.steps // 2), args.warmup)
            extra[cfg] = result_entry(r, max(5, args.steps // 2))
            del r
            torch.cuda.empty_cache()
        line["configs"] = extra

    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        D.barrier(dist)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
