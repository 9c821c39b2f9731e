#!/usr/bin/env python3
"""Benchmark: Internet-checksum GiB/s, device-resident, on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]

--gpus N > 1 without a launcher starts N rank processes itself (one per GPU,
torchrun's environment); under torchrun WORLD_SIZE must equal N.  Either way
rank r times its own slice and the line reports the max over ranks.

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
_T0 = time.perf_counter()  # process start, for the line's wall-time figure
DRIVER_LIMIT_S = 600  # the driver's per-run limit an N-GPU run must fit
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip table)
METRIC = "Internet-checksum GiB/s (device-resident), 1500B & 64KB packet batches"


def _host(t):
    """A device tensor's values as numpy, copied through pinned memory only
    (tcp_amd.to_host)."""
    from tcp_amd import to_host
    return to_host(t)


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
    ap.add_argument("--settle-ms", type=float, default=300.0,
                    help="untimed: the warm-up also lasts at least this long (GPU clocks out of idle "
                         "whatever W is; 0 = exactly W launches).  300: with 30 one box read the headline "
                         "at 0.908 against 0.935 with 300 in the same call, and the secondary configs "
                         "1-2.5 %% low (profiles/r04/gap/)")
    ap.add_argument("--arena-policy", choices=("free", "keep", "prealloc"), default="prealloc",
                    help="secondary configs' arenas: allocated and filled all before the first is timed (default), "
                         "kept, or freed after each config (round 4's: the config timed right after the 16-GiB "
                         "TSO arena was freed read 1.4-3.3 %% slow while the driver released it, "
                         "profiles/r05/order/)")
    ap.add_argument("--child-gap-ms", type=float, default=0.0,
                    help="measurement: idle time after the PMC / trace children exit, before this process "
                         "allocates (a 2-s pause changed nothing for the headline: 0.9400-0.9409 with it, "
                         "0.9386-0.9407 without, 0.9399-0.9402 with no children; profiles/r05/order/)")
    ap.add_argument("--gap-ms", type=float, default=0.0,
                    help="measurement: idle time between the secondary configs")
    ap.add_argument("--no-pmc", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-kind", choices=("reference", "port"), default="reference",
                    help="CPU baseline: the reference's own checksum_peso (oracle/_ref) or the oracle's port")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--trace-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--e2e-multi-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--no-trace", action="store_true", help="skip the rocprofv3 kernel-trace child")
    ap.add_argument("--knob", action="append", default=[], metavar="KEY=VALUE",
                    help="measurement only: a libtcsum debug knob (include/tcsum_debug.h) set for the whole run, "
                         "its PMC and trace children included; the line records it")
    ap.add_argument("--cpu-rehearsal", action="store_true",
                    help="rehearse the N-rank launcher, rendezvous, barrier and max-over-ranks timing on CPU "
                         "(gloo, a numpy stand-in for the kernel; no GPU, no GPU numbers)")
    return ap.parse_args()


def algorithmic_split(batch):
    """(bytes read, bytes written) of algorithmic_bytes: every packet byte and
    its descriptor read; the result (or, tx fill, the 2 x 2-byte checksum
    fields written into the packet) written."""
    desc = 24 if batch.kind == "peso" else 16
    if batch.kind == "peso":
        wr = 2
    else:
        wr = {"sums": 4, "tx": 4, "rx": 1, "txo": 4 + 1}[batch.op]
    return batch.total_bytes + desc * batch.n, wr * batch.n


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


# Counter bytes per byte of each access class the step kernels make, measured
# by scripts/pmc_calib.py on MI355X (known byte counts, each class alone after
# an L2 flush; profiles/r03/pmc_calib.json, profiles/history/DESIGN_rounds1-5.md §6).  Keys: the class
# kernels of scripts/pmc_calib.hip; None would fall back to the guide's
# blanket x2 for FETCH_SIZE.
PMC_CALIB = {
    "k_stream<true>": 0.5, "k_stream<false>": 0.5,            # 128-B requests tallied at 64 B (the guide's x2)
    "k_desc<16>": 0.5004, "k_desc<24>": 0.5002,                # lane groups on dense records: the same
    "k_sparse16@1500": 4.0008, "k_sparse16@4532": 4.0013,      # one 64-B request per lone 16-B chunk
    "k_load<unsigned int, 4>": 0.5006, "k_load<unsigned long, 16>": 1.0012,
    "k_store_dense<unsigned char>": 1.0, "k_store_dense<unsigned short>": 1.0,
    "k_store_dense<unsigned int>": 1.0, "k_store_dense<unsigned long>": 1.0,
    "k_store_wg16": 8.0,                                       # 16 B per lone u16
    "k_store_field<1>": 16.0, "k_store_field<2>": 15.3591,     # 32 B per lone 2-B field
}


def access_classes(batch) -> dict:
    """Bytes one step moves per access class: (calibration class, counter) ->
    bytes.  Every packet byte is one streaming 16-B-per-lane nontemporal read;
    descriptors are read by lane groups; results are dense stores; the
    deferred tx fill adds its scratch (8 B per packet written, then read by
    k_tx_scatter with the descriptor offsets) and the scattered field writes."""
    n = batch.n
    c = {("k_stream<true>", "FETCH_SIZE"): batch.total_bytes}
    if batch.kind == "peso":
        c[("k_desc<24>", "FETCH_SIZE")] = 24 * n
        # one u16 per range; consecutive ranges' workgroups share an XCD (xcd_block), so
        # their results merge in its L2 like a dense store (k_store_wg16's 16 B per
        # store is the round-robin case)
        c[("k_store_dense<unsigned short>", "WRITE_SIZE")] = 2 * n
        return c
    c[("k_desc<16>", "FETCH_SIZE")] = 16 * n
    if batch.op == "sums":
        c[("k_store_dense<unsigned int>", "WRITE_SIZE")] = 4 * n
    elif batch.op == "rx":
        c[("k_store_dense<unsigned char>", "WRITE_SIZE")] = n
    elif batch.op == "txo":
        c[("k_store_dense<unsigned int>", "WRITE_SIZE")] = 4 * n
        c[("k_store_dense<unsigned char>", "WRITE_SIZE")] = n
    else:  # tx, deferred: fill (values + positions) -> k_tx_scatter
        c[("k_store_dense<unsigned long>", "WRITE_SIZE")] = 8 * n
        c[("k_load<unsigned int, 4>", "FETCH_SIZE")] = 8 * n
        c[("k_load<unsigned long, 16>", "FETCH_SIZE")] = 8 * n
        c[("k_store_field<2>", "WRITE_SIZE")] = 4 * n  # IPv4 + TCP/UDP field: every synthetic packet has both
    return c


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
KNOBS: list = []  # --knob KEY=VALUE (measurement), passed on to the profiler children


def time_config(torch, tc, workload, config, rank, steps, warmup, dist=None, probes=True, pre=None):
    """pre: (batch, arena, descs) materialized beforehand (--arena-policy prealloc)."""
    if pre is not None:
        batch, arena, descs = pre
    else:
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
    # untimed for the line: the same K launches again, each between its own
    # pair of events -- the per-launch median the rocprof trace is compared with
    pairs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for e0, e1 in pairs:
        e0.record(stream)
        launch(tc, batch, arena, descs, out, flags)
        e1.record(stream)
    torch.cuda.synchronize()
    per_launch = sorted(e0.elapsed_time(e1) for e0, e1 in pairs)
    r = dict(batch=batch, arena=arena, descs=descs, out=out, flags=flags, ms=ms, wall_s=wall, steps=steps,
             launch_median_ms=per_launch[len(per_launch) // 2])
    if probes:
        run_probes(torch, tc, r)
    return r


def run_probes(torch, tc, r) -> None:
    """The probes, after the timed region (and after self_check: the tx probe
    leaves the batch's checksum fields junk)."""
    batch, arena, descs, out, flags = r["batch"], r["arena"], r["descs"], r["out"], r["flags"]
    r["probes"] = probe_compare(torch, tc, batch, lambda: launch(tc, batch, arena, descs, out, flags), arena,
                                r["steps"], descs=descs)


def probe_compare(torch, tc, batch, product, arena, steps, rounds=5, descs=None):
    """The roofline's achievable side, measured beside the product kernel
    (after the timed region, never inside it): rounds of [product x m, plain
    read x m, tile-shaped reads x m] launches, each with its own events, so
    they see the same clocks and the same HBM state; per-launch medians.
    Plain read: k_probe_read<4>, contiguous 1 KiB per load instruction.  Tile
    read: k_probe_tile in the product's own geometry (lanes x loads, XCD
    order) over the same bytes -- the product minus descriptors and sums;
    tile_dep: the same with each unit's loads behind one dependent 16-B read,
    as the product's loads wait for its descriptor.  segments (checksum_peso
    batches): tcsum_probe_segments -- the product's own descriptors, lanes,
    loads, edge policy and block order with the arithmetic and the store
    removed, priced on the same algorithmic bytes as the product.
    achievable = the fastest."""
    g, u = tc.pick_geometry(batch.total_bytes // max(batch.n, 1))
    sink = torch.zeros(1, dtype=torch.uint32, device=arena.device)
    nbytes = batch.arena_bytes
    tile_ok = True
    try:
        tc.probe_tile(arena, nbytes, g, u, sink)
    except RuntimeError:
        tile_ok = False
    kinds = {"product": product, "read": lambda: tc.probe_read(arena, nbytes, sink)}
    if tile_ok:
        kinds["tile"] = lambda: tc.probe_tile(arena, nbytes, g, u, sink)

        # each unit's loads behind one dependent 16-B read, like the product's descriptor
        kinds["tile_dep"] = lambda: tc.probe_tile(arena, nbytes, g, u, sink, dep=True)
    if batch.kind == "peso" and descs is not None:
        kinds["segments"] = lambda: tc.probe_segments(arena, descs, batch.n, batch.total_bytes, sink)
    elif descs is not None:
        kinds["segments"] = lambda: tc.probe_ipv4(arena, descs, batch.n, batch.total_bytes, rx=batch.op == "rx",
                                                  sink=sink)
        if batch.op == "tx":  # the ceiling for a kernel that must write: the same loads + the fill's own writes
            kinds["segments_tx"] = lambda: tc.probe_ipv4(arena, descs, batch.n, batch.total_bytes, tx=True,
                                                         sink=sink)
            # the design-independent floor: one plain read of the bytes + the
            # same 2 field writes per packet, stores in-stream or deferred
            fh = tc.txfloor_prepare(arena, nbytes, descs, batch.n, batch.total_bytes)
            kinds["floor_instream"] = lambda: tc.probe_txfloor(fh, deferred=False)
            kinds["floor_deferred"] = lambda: tc.probe_txfloor(fh, deferred=True)
            # deferred, each field's dword loaded before its store (the product's form)
            kinds["floor_warm"] = lambda: tc.probe_txfloor(fh, variant=11)
    m = max(2, steps // rounds)
    stream = torch.cuda.current_stream()
    per = {k: [] for k in kinds}
    for _ in range(rounds):
        for k, fn in kinds.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            fn()  # one untimed launch: the previous kind's tail is not charged here
            e0.record(stream)
            for _ in range(m):
                fn()
            e1.record(stream)
            torch.cuda.synchronize()
            per[k].append(e0.elapsed_time(e1) / m)
    med = {k: sorted(v)[len(v) // 2] for k, v in per.items()}
    res = {"product_ms": med["product"], "read_gbs": nbytes / (med["read"] * 1e-3) / 1e9,
           "geometry": [g, u], "rounds": rounds, "launches_per_round": m}
    if tile_ok:
        res["tile_gbs"] = nbytes / (med["tile"] * 1e-3) / 1e9
        res["tile_dep_gbs"] = nbytes / (med["tile_dep"] * 1e-3) / 1e9
    if "segments" in med:
        res["segments_gbs"] = algorithmic_bytes(batch) / (med["segments"] * 1e-3) / 1e9
    if "segments_tx" in med:
        res["segments_tx_gbs"] = algorithmic_bytes(batch) / (med["segments_tx"] * 1e-3) / 1e9
    for k in ("floor_instream", "floor_deferred", "floor_warm"):
        if k in med:
            res[k + "_gbs"] = algorithmic_bytes(batch) / (med[k] * 1e-3) / 1e9
    return res


def result_entry(r, steps):
    b = r["batch"]
    ms_step = r["ms"] / steps
    alg = algorithmic_bytes(b)
    ach = alg / (ms_step * 1e-3) / 1e9
    p = r["probes"]
    best = max(p["read_gbs"], p.get("tile_gbs", 0.0), p.get("tile_dep_gbs", 0.0), p.get("segments_gbs", 0.0))
    side = alg / (p["product_ms"] * 1e-3) / 1e9  # the product in the interleaved rounds
    # a kernel that writes is priced against the tx floor: the fastest of one
    # plain read + the same field writes, in-stream, deferred, or deferred
    # with each field's dword loaded first
    floor = max(p.get("floor_instream_gbs", 0.0), p.get("floor_deferred_gbs", 0.0), p.get("floor_warm_gbs", 0.0))
    ceil = floor if floor > 0 else best
    entry = {
        "workload": b.config,
        "packets": b.n,
        "payload_bytes": b.total_bytes,
        "gib_s": b.total_bytes / (ms_step * 1e-3) / GIB,
        "ms_per_step": ms_step,
        "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(ach / HBM_PEAK_GBS, 4),
                     "achievable_read": round(best, 1),
                     "achievable": round(ceil, 1),
                     "achievable_kind": "tx floor (one plain read + the fill's 2 field writes per packet, "
                                        "fastest of in-stream / deferred / deferred after loading each "
                                        "field's dword)" if floor > 0 else "fastest read probe",
                     "frac_of_achievable": round(side / ceil, 4),
                     "probes": {"plain_read_gbs": round(p["read_gbs"], 1),
                                "tile_read_gbs": round(p["tile_gbs"], 1) if "tile_gbs" in p else None,
                                "tile_dep_read_gbs": round(p["tile_dep_gbs"], 1) if "tile_dep_gbs" in p else None,
                                "segments_read_gbs": round(p["segments_gbs"], 1) if "segments_gbs" in p else None,
                                "segments_tx_gbs": round(p["segments_tx_gbs"], 1) if "segments_tx_gbs" in p else None,
                                "floor_instream_gbs": round(p["floor_instream_gbs"], 1)
                                if "floor_instream_gbs" in p else None,
                                "floor_deferred_gbs": round(p["floor_deferred_gbs"], 1)
                                if "floor_deferred_gbs" in p else None,
                                "floor_warm_gbs": round(p["floor_warm_gbs"], 1) if "floor_warm_gbs" in p else None,
                                "tile_geometry": p["geometry"], "product_gbs_same_rounds": round(side, 1),
                                "rounds": p["rounds"], "launches_per_round": p["launches_per_round"]}},
    }
    return entry


# ------------------------------------------------------------ PMC traffic

def is_step_kernel(name: str) -> bool:
    """The kernels one bench step launches (the probes are not among them)."""
    return "k_segments" in name or "k_ipv4<" in name or "k_tx_scatter" in name or "k_flat_" in name


def step_counter(files, counter: str):
    """One step's value of `counter` from rocprofv3 counter-collection CSVs:
    per step kernel the median over its launches, summed over the kernels a
    step launches (tx fill: k_ipv4 + k_tx_scatter).  Only kernels launched
    every step count: rx's setup runs one tx fill (a k_ipv4 of another shape +
    k_tx_scatter) that is no part of its step.  None without a step kernel."""
    per = {}  # kernel name -> values
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                if is_step_kernel(name) and row.get("Counter_Name", counter) == counter:
                    per.setdefault(name.split("(")[0], []).append(float(row["Counter_Value"]))
    if not per:
        return None
    top = max(len(v) for v in per.values())
    return sum(sorted(v)[len(v) // 2] for v in per.values() if len(v) == top)


def pmc_traffic(config: str):
    """HBM bytes per launch from rocprofv3 counters, in separate passes
    (FETCH_SIZE, then WRITE_SIZE), run as a child before this process touches
    the GPU.  gfx950: FETCH_SIZE counts half the bytes of a wide streaming read
    (MI355X_MICROARCH.md §HBM) -> x2; both counters are in KiB."""
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None, "rocprofv3 not found", None
    vals = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix=f"tcsum_pmc_{counter}_")
        cmd = [prof, "--pmc", counter, "--output-format", "csv", "-d", d, "-o", "pmc", "--",
               sys.executable, os.path.abspath(__file__), "--pmc-child", "--config", config,
               "--steps", "3", "--warmup", "1"] + [f"--knob={k}" for k in KNOBS]
        try:
            subprocess.run(cmd, check=True, timeout=240, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                           env=dict(os.environ, TMPDIR=d))
        except (subprocess.SubprocessError, OSError) as e:
            return None, f"rocprofv3 {counter} pass failed: {type(e).__name__}", None
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        keep = os.environ.get("TCSUM_PMC_KEEP")  # directory to keep the raw counter CSVs in
        if keep:
            os.makedirs(keep, exist_ok=True)
            for i, f in enumerate(files):
                shutil.copy(f, os.path.join(keep, f"pmc_{counter.lower()}_{config}{'_%d' % i if i else ''}.csv"))
        v = step_counter(files, counter)
        shutil.rmtree(d, ignore_errors=True)
        if v is None:
            return None, f"no {counter} rows for the checksum kernel", None
        vals[counter] = v
    raw = {k: v * 1024 for k, v in vals.items()}  # KiB -> bytes, as the counters report them
    from tcp_amd import workload
    batch = workload.make_batch(config)
    if PMC_CALIB is None:
        traffic = raw["FETCH_SIZE"] * 2 + raw["WRITE_SIZE"]
        return traffic, None, {"raw": raw, "method": "blanket x2 on FETCH_SIZE (uncalibrated)",
                               "raw_bytes": raw_traffic(batch, raw)}
    traffic, detail = calibrated_traffic(access_classes(batch), raw)
    return traffic, None, {"per_counter": detail, "method": "per access class (scripts/pmc_calib.py)",
                           "raw_bytes": raw_traffic(batch, raw)}


def raw_traffic(batch, raw: dict) -> dict:
    """The counters with the guide's gfx950 corrections only (MI355X_MICROARCH.md,
    HBM / rocprofv3: FETCH_SIZE x 2, WRITE_SIZE as is), in bytes per step, and
    each over the algorithmic bytes of its direction.  Unlike the calibrated
    `traffic`, nothing here is divided by what an access class costs on its
    own, so write amplification (a lone 2-byte field costing a 32-B or 64-B
    write) and re-fetched lines show as they are."""
    rd, wr = algorithmic_split(batch)
    fetch = raw["FETCH_SIZE"] * 2
    write = raw["WRITE_SIZE"]
    # the bytes the step's kernels store by design (the deferred tx fill also
    # writes 8 B of scratch per packet): amplification over those is the
    # hardware's, over the algorithmic writes the design's and the hardware's
    cls = access_classes(batch)
    nominal_wr = sum(v for (_, c), v in cls.items() if c == "WRITE_SIZE")
    return {"fetch_bytes": round(fetch), "write_bytes": round(write), "total_bytes": round(fetch + write),
            "algorithmic_read_bytes": rd, "algorithmic_write_bytes": wr, "step_store_bytes": nominal_wr,
            "fetch_vs_algorithmic_read": round(fetch / rd, 4) if rd else None,
            "write_vs_algorithmic_write": round(write / wr, 4) if wr else None,
            "write_vs_step_stores": round(write / nominal_wr, 4) if nominal_wr else None,
            "total_vs_algorithmic": round((fetch + write) / (rd + wr), 4),
            "method": "FETCH_SIZE x 2 + WRITE_SIZE (KiB x 1024), the guide's corrections only"}


def calibrated_traffic(classes: dict, raw: dict):
    """Per counter: the bytes the step's classes move, scaled by how far the
    raw counter is from what those classes report on their own (PMC_CALIB)."""
    traffic, detail = 0.0, {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        nominal = sum(b for (k, c), b in classes.items() if c == counter)
        expect = sum(b * PMC_CALIB[k] for (k, c), b in classes.items() if c == counter)
        ratio = raw[counter] / expect if expect else 1.0
        traffic += nominal * ratio
        detail[counter] = {"raw": round(raw[counter]), "expected_raw": round(expect), "nominal": nominal,
                           "measured_vs_expected": round(ratio, 4)}
    return traffic, detail


def rocprof_trace(config: str, steps: int, warmup: int, settle_ms: float):
    """The dominant kernel's launch durations from `rocprofv3 --kernel-trace
    --stats` of this same bench (one config, same K/W/settle), run as a child
    before this process touches the GPU: (median_ns, mean_ns, launches,
    kernel name).  Only the full-size launches count (the largest grid of the
    checksum kernel), i.e. the warm-up, settle and timed launches."""
    prof = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(prof):
        return None, "rocprofv3 not found"
    d = tempfile.mkdtemp(prefix="tcsum_trace_")
    cmd = [prof, "--kernel-trace", "--stats", "--output-format", "csv", "-d", d, "-o", "trace", "--",
           sys.executable, os.path.abspath(__file__), "--pmc-child", "--trace-child", "--config", config,
           "--steps", str(steps), "--warmup", str(warmup), "--settle-ms", str(settle_ms)] + \
        [f"--knob={k}" for k in KNOBS]
    try:
        res = subprocess.run(cmd, check=True, timeout=300, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                             env=dict(os.environ, TMPDIR=d), text=True)
    except (subprocess.SubprocessError, OSError) as e:
        shutil.rmtree(d, ignore_errors=True)
        return None, f"rocprofv3 kernel-trace pass failed: {type(e).__name__}"
    child = {}
    for ln in res.stdout.splitlines():
        if ln.startswith("{") and "child_ms_per_step" in ln:
            child = json.loads(ln)
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    keep = os.environ.get("TCSUM_PMC_KEEP")
    if keep:
        os.makedirs(keep, exist_ok=True)
        for f in files + glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
            shutil.copy(f, os.path.join(keep, f"trace_{config}_{os.path.basename(f)}"))
    rows = []
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                if is_step_kernel(name):
                    rows.append((name, int(row["Grid_Size_X"]),
                                 int(row["End_Timestamp"]) - int(row["Start_Timestamp"])))
    shutil.rmtree(d, ignore_errors=True)
    if not rows:
        return None, "no checksum-kernel rows in the trace"
    total = {}
    for name, grid, dur in rows:
        total[name] = total.get(name, 0) + dur

    def median_at_full_grid(name):
        grid = max(g for n, g, _ in rows if n == name)
        return sorted(dur for n, g, dur in rows if n == name and g == grid)

    name = max(total, key=total.get)
    durs = median_at_full_grid(name)
    # every kernel of a step (tx fill: the fill + k_tx_scatter), median each
    step_ns = sum(median_at_full_grid(k)[len(median_at_full_grid(k)) // 2] for k in total)
    return (durs[len(durs) // 2], sum(durs) / len(durs), len(durs), name, step_ns, len(total), child), None


# ------------------------------------------------------------ CPU baseline

def cpu_model():
    """The GPU box's host CPU as /proc/cpuinfo names it: model, logical CPUs,
    sockets, NUMA nodes."""
    try:
        with open("/proc/cpuinfo") as f:
            lines = f.readlines()
        names = [ln.split(":", 1)[1].strip() for ln in lines if ln.startswith("model name")]
        sockets = len({ln.split(":", 1)[1].strip() for ln in lines if ln.startswith("physical id")})
        nodes = len(glob.glob("/sys/devices/system/node/node[0-9]*"))
        return (f"{names[0]} ({len(names)} logical CPUs on the host, {sockets or '?'} socket(s), "
                f"{nodes or '?'} NUMA node(s))") if names else None
    except OSError:
        return None


def _cpuset_count(text):
    """Logical CPUs in a cpuset list such as "0-15,32-47"."""
    n = 0
    for part in text.strip().split(","):
        if part:
            a, _, b = part.partition("-")
            n += int(b or a) - int(a) + 1
    return n


def cpu_allowance(base="/sys/fs/cgroup", proc_cgroup="/proc/self/cgroup"):
    """The CPUs this process may actually use, which on a shared GPU box is not
    os.cpu_count() (the whole host): the affinity mask, and the cgroup's
    cpuset and CPU quota (v2 cpu.max, or v1 cfs_quota_us / cfs_period_us).
    `effective` = the smallest of them (a quota of 16.0 CPUs means at most
    16 threads' worth of CPU time however many threads run)."""
    import math
    out = {"host_logical": os.cpu_count()}
    try:
        out["affinity"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        pass
    v2, v1 = "", {}
    try:
        with open(proc_cgroup) as f:
            for ln in f:
                h, ctl, path = ln.strip().split(":", 2)
                if h == "0" and not ctl:
                    v2 = path
                for c in ctl.split(","):
                    if c:
                        v1[c] = path
    except (OSError, ValueError):
        pass
    quotas, cpusets = [], []

    def walk(root, rel):  # the process's own cgroup and each ancestor: the tightest limit binds
        d = os.path.normpath(root + rel) if rel and rel != "/" else root
        while d.startswith(root):
            yield d
            if d == root:
                break
            d = os.path.dirname(d)

    def read(path):
        try:
            with open(path) as f:
                return f.read().strip()
        except OSError:
            return ""

    for d in walk(base, v2):  # cgroup v2
        t = read(os.path.join(d, "cpu.max")).split()
        if len(t) == 2 and t[0] != "max":
            quotas.append(int(t[0]) / int(t[1]))
        t = read(os.path.join(d, "cpuset.cpus.effective"))
        if t:
            cpusets.append(_cpuset_count(t))
    if "cpu" in v1:  # cgroup v1
        for root in (f"{base}/cpu", f"{base}/cpu,cpuacct"):
            for d in walk(root, v1["cpu"]):
                q, per = read(os.path.join(d, "cpu.cfs_quota_us")), read(os.path.join(d, "cpu.cfs_period_us"))
                if q and per and int(q) > 0:
                    quotas.append(int(q) / int(per))
    if "cpuset" in v1:
        for d in walk(f"{base}/cpuset", v1["cpuset"]):
            t = read(os.path.join(d, "cpuset.effective_cpus")) or read(os.path.join(d, "cpuset.cpus"))
            if t:
                cpusets.append(_cpuset_count(t))
    if quotas:
        out["cpu_quota"] = round(min(quotas), 2)
    if cpusets:
        out["cpuset"] = min(cpusets)
    lim = [v for v in (out.get("affinity"), out.get("cpuset")) if v]
    if quotas:
        lim.append(max(1, math.floor(min(quotas))))
    out["effective"] = min(lim) if lim else (os.cpu_count() or 1)
    return out


def cpu_baseline(torch, r, seconds, kind="reference", cache_sample=True):
    """The reference's checksum_peso (oracle/_ref/libtcpref.so, compiled from
    /root/reference; kind "port" = the oracle's restatement) on the same
    segments in host memory, timed on this host's cores:

      value      1 thread -- the reference checksums on its single work_thread
                 (exmsg.c:123) -- over a DRAM-resident sample (>= 1 GiB of the
                 batch, larger than any L3; re-summed for >= `seconds`);
      value_all  as many threads as this process's CPU allowance holds
                 (cpu_allowance: affinity, cgroup cpuset and quota -- on a
                 shared box far fewer than the host's os.cpu_count()), same
                 sample, with each thread's own rate (min / median / max);
      cache_resident  both, over a ~100 MB sample that fits the host's L3.

    cache_sample=False (the secondary configs): the DRAM sample only.
    A requested "reference" that is not built fails (no silent fallback)."""
    from oracle import pyoracle
    import numpy as np
    pyoracle.build()
    b = r["batch"]

    def sample(max_bytes):
        lens = b.descs["len"].astype(np.int64)
        n = int(np.searchsorted(np.cumsum(lens), max_bytes)) + 1
        n = max(1, min(b.n, n))
        end = int(b.descs["offset"][n - 1] + b.descs["len"][n - 1])
        host = _host(r["arena"][: end + 16])
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
        return host, segs, want, n

    allow = cpu_allowance()
    threads_all = min(256, allow["effective"])  # orc_time_peso runs at most 256 threads
    res = {"unit": "GiB/s", "kind": kind, "cores": 1, "cores_all": os.cpu_count(), "cores_effective": threads_all,
           "cpu_allowance": allow, "host_cpu": cpu_model(),
           "placement": "each timing thread pinned to its own logical CPU, its slice of the sample copied "
                        "(first-touched) by that thread before the timed region: NUMA-local"}
    what = "segments" if b.kind == "peso" else "packets' L4 ranges"
    big = min(b.total_bytes, 1 << 30)
    legs = [("dram", big, seconds)] + ([("cache", 96 << 20, seconds / 2)] if cache_sample else [])
    for label, nbytes, secs in legs:
        host, segs, want, n = sample(nbytes)
        rate1, got_kind, cs1 = pyoracle.time_peso(host, segs, 1, secs, kind=kind)
        rate_all, _, cs_all, per = pyoracle.time_peso(host, segs, threads_all, max(2.0, secs / 2), kind=kind,
                                                     thread_rates=True)
        per = sorted(per)
        part = {"value": round(rate1 / GIB, 3), "value_all": round(rate_all / GIB, 3),
                "threads_all": threads_all, "scaling_all": round(rate_all / rate1, 2) if rate1 else None,
                "per_thread_all": {"min": round(per[0] / GIB, 3), "median": round(per[len(per) // 2] / GIB, 3),
                                   "max": round(per[-1] / GIB, 3)},
                "sample_bytes": int(segs["len"].sum()),
                "sample": f"first {n} {what} of the {b.config} batch ({int(segs['len'].sum()) / 1e6:.0f} MB), "
                          f"re-summed for >= {secs:.0f} s (1 thread) / {max(2.0, secs / 2):.0f} s "
                          f"({threads_all} threads)",
                "parity": bool(cs1 == want and cs_all == want)}
        if label == "dram" and cache_sample and kind == "reference":
            # BASELINE.md's optional strong-CPU line: the reference at -O3 with AVX2
            s1, _, c1 = pyoracle.time_peso(host, segs, 1, secs / 2, kind="reference_o3")
            s_all, _, c_all = pyoracle.time_peso(host, segs, threads_all, 2.0, kind="reference_o3")
            part["strong_cpu"] = {"flags": "-O3 -march=x86-64-v3", "value": round(s1 / GIB, 3),
                                  "value_all": round(s_all / GIB, 3), "parity": bool(c1 == want and c_all == want)}
        del host
        if label == "dram":
            res.update(part)
        else:
            res["cache_resident"] = part
    return res


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
        host[:] = _host(r["arena"][:nbytes])
        out = np.zeros(b.n, np.uint16)
        tc.host_batch_peso(host, b.descs)  # warm (allocates device buffers)
        t0 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            out = tc.host_batch_peso(host, b.descs)
        dt = (time.perf_counter() - t0) / reps
        same = bool((out == _host(r["out"])).all())
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
               "path": "pinned host -> hipMemcpyAsync H2D (the first 64 MiB before the rest of the descriptors are read, then chunks of a quarter of the batch, in order on one copy stream; 16-B descriptors; kernels on a second stream behind per-chunk events) -> kernel -> D2H",
               "h2d_copy_gib_s": round(link, 2),
               "matches_device_resident": same}
        ndev = torch.cuda.device_count()
        if ndev > 1:  # the same host batch sharded over every GPU of the node, in a child with a time limit
            res["multi_device"] = e2e_multi_child(b.config, ndev)
    finally:
        L.tcsum_host_free(p)
    try:
        res["host_queue_rx"] = e2e_host_queue_rx(torch, tc)
    except Exception as e:  # reported, never fatal
        res["host_queue_rx"] = {"error": repr(e)}
    return res


def e2e_host_queue_rx(torch, tc):
    """The receive path from host memory (the frames plat/netif_pcap.c hands
    the stack): configs[3]'s 1M IPv4 frames in pinned host memory ->
    tcsum_host_batch_ipv4_rx_verify (copy-engine pieces, k_ipv4 rx) ->
    verdicts; checked against the device-resident verdicts."""
    from tcp_amd import workload
    b = workload.make_batch("mixed_rx")
    arena, descs = workload.materialize(b)
    want, _ = tc.batch_ipv4_rx_verify(arena, descs, b.n, b.total_bytes, want_flags=False)
    want = _host(want)
    ha = tc.HostArena(arena.numel())
    try:
        ha.array[:] = _host(arena)
        del arena, descs
        torch.cuda.empty_cache()
        v, _, _ = tc.host_batch_ipv4_rx_verify(ha, b.descs)  # warm (device buffers)
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            v, _, _ = tc.host_batch_ipv4_rx_verify(ha, b.descs)
        dt = (time.perf_counter() - t0) / reps
        return {"gib_s": round(b.total_bytes / dt / GIB, 2), "ms_per_batch": round(dt * 1e3, 2), "frames": b.n,
                "path": "pinned host frames -> copy-engine pieces into HBM -> k_ipv4 rx verify -> verdicts to host",
                "matches_device_resident": bool((v == want).all())}
    finally:
        ha.free()


def e2e_multi_child(config: str, ndev: int, timeout_s: float = 240.0):
    """tcsum_host_batch_peso_multi over every GPU of the node, measured in a
    child process (`bench.py --e2e-multi-child`) so that a first run of the
    cross-device path on a new node can only cost this field, never the bench
    line: the child is killed after timeout_s."""
    cmd = [sys.executable, os.path.abspath(__file__), "--e2e-multi-child", "--config", config]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout_s)
    except subprocess.TimeoutExpired:
        return {"gpus": ndev, "error": f"timed out after {timeout_s:.0f} s"}
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"gpus": ndev, "error": f"rc {r.returncode}: {r.stderr[-300:]}"}
    return json.loads(lines[-1])


def shard_report(shards: list, identity) -> dict:
    """Per shard of a multi-device host batch (tcsum_debug_shards): the
    device that took it, named as the device-resident line names its ranks'
    GPUs, and that shard's own packets, bytes, wall time and rate, plus the
    spread of the shard times -- a slow host link or GPU then shows as its
    own entry instead of a lower aggregate."""
    rows = [{"device": identity(s["device"]), "packets": s["count"], "bytes": s["bytes"], "rc": s["rc"],
             "ms": round(s["ms"], 3),
             "gib_s": round(s["bytes"] / (s["ms"] * 1e-3) / GIB, 2) if s["ms"] > 0 else None} for s in shards]
    ms = [r["ms"] for r in rows if r["packets"]] or [0.0]
    return {"shards": rows, "devices": [r["device"] for r in rows],
            "shard_ms_spread": {"min": min(ms), "max": max(ms), "max_over_min": round(max(ms) / max(1e-9, min(ms)), 4)}}


def e2e_multi_main(config: str) -> None:
    """The child: the batch generated on GPU 0, copied to pinned host memory,
    then checksummed from there by every GPU (one shard each) and checked
    against the device-resident results; the same for configs[3]'s frames
    through the host-queue rx verify.  Every shard's device and time is
    reported."""
    import ctypes
    import numpy as np
    import torch
    import tcp_amd as tc
    from tcp_amd import _lib, workload
    devs = list(range(torch.cuda.device_count()))
    ident = lambda d: device_identity(torch, d)  # noqa: E731
    b = workload.make_batch(config)
    arena, descs = workload.materialize(b)
    want = _host(tc.batch_peso(arena, descs, b.n, b.total_bytes))
    L = _lib.lib()
    p = L.tcsum_host_alloc(b.alloc_bytes)
    if not p:
        raise MemoryError("tcsum_host_alloc")
    res = {"gpus": len(devs)}
    try:
        host = np.ctypeslib.as_array((ctypes.c_uint8 * b.alloc_bytes).from_address(p))
        host[:] = _host(arena[: b.alloc_bytes])
        del arena, descs
        torch.cuda.empty_cache()
        out = tc.host_batch_peso_multi(host, b.descs, devs)
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            out = tc.host_batch_peso_multi(host, b.descs, devs)
        dt = (time.perf_counter() - t0) / reps
        res.update({"gib_s": round(b.total_bytes / dt / GIB, 2), "matches_device_resident": bool((out == want).all())})
        res.update(shard_report(tc.last_shards(), ident))  # the last repetition's shards
    finally:
        L.tcsum_host_free(p)
    try:  # the receive path's host-queue batch over the same devices
        rb = workload.make_batch("mixed_rx")
        arena, descs = workload.materialize(rb)
        wv, _ = tc.batch_ipv4_rx_verify(arena, descs, rb.n, rb.total_bytes, want_flags=False)
        wv = _host(wv)
        ha = tc.HostArena(arena.numel())
        try:
            ha.array[:] = _host(arena)
            del arena, descs
            torch.cuda.empty_cache()
            v, _, _ = tc.host_batch_ipv4_rx_verify(ha, rb.descs, devices=devs)
            t0 = time.perf_counter()
            for _ in range(reps):
                v, _, _ = tc.host_batch_ipv4_rx_verify(ha, rb.descs, devices=devs)
            dt = (time.perf_counter() - t0) / reps
            q = {"frames": rb.n, "gib_s": round(rb.total_bytes / dt / GIB, 2),
                 "matches_device_resident": bool((v == wv).all())}
            q.update(shard_report(tc.last_shards(), ident))
            res["host_queue_rx"] = q
        finally:
            ha.free()
    except Exception as e:  # reported, never fatal
        res["host_queue_rx"] = {"error": repr(e)}
    print(json.dumps(res), flush=True)


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
    for served in (False, True):  # one launch + its wait per call / the call server's resident wave
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
    res["note"] = ("plain: one launch per call, the host spinning on a completion word the stream writes behind "
                   "it; served_: tcsum_call_server (one resident wave polling pinned memory). Use the batch API "
                   "for throughput")
    return res


SELF_CHECK_N = 4096  # segments per rank re-summed after the timed region


def device_identity(torch, dev: int) -> dict:
    """Which GPU this rank timed: its HIP ordinal and PCI address (RCCL runs
    one rank per GPU; two ranks on one device would double-count it)."""
    p = torch.cuda.get_device_properties(dev)
    pci = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}"
    return {"ordinal": dev, "pci": pci, "uuid": str(p.uuid), "name": p.name,
            "visible": os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES")}


def self_check(torch, tc, workload, head, seed: int) -> dict:
    """Re-sum a seeded sample of this rank's own segments in a separate,
    smaller launch and compare with what the timed launches produced: a
    self-consistency check that needs no oracle on the box (the oracle
    parity lives in tests/).  The tx fill writes into the packets, so for it
    the sample is filled again and must come out byte-identical
    (idempotence)."""
    import numpy as np
    b, arena, out = head["batch"], head["arena"], head["out"]
    n = min(SELF_CHECK_N, b.n)
    idx = np.sort(np.random.default_rng(seed).choice(b.n, size=n, replace=False))
    sub = tc.descs_to_device(b.descs[idx], arena.device)
    if b.op == "tx":
        lens = np.minimum(b.descs["len"][idx].astype(np.int64), 78)  # the fill writes only there
        offs = b.descs["offset"][idx].astype(np.int64)
        pos = torch.from_numpy(np.concatenate([o + np.arange(k) for o, k in zip(offs, lens)])).pin_memory().to(arena.device)
        before = _host(arena[pos])
        tc.batch_ipv4_tx_fill(arena, sub, n, 0, want_flags=False)
        bad = int((_host(arena[pos]) != before).sum())
        return {"segments": n, "mismatches": bad}
    if b.kind == "peso":
        got = tc.batch_peso(arena, sub, n, 0)
    elif b.op == "rx":
        got, _ = tc.batch_ipv4_rx_verify(arena, sub, n, 0, want_flags=False)
    elif b.op == "txo":
        got, _ = tc.batch_ipv4_tx_offload(arena, sub, n, 0)
    else:
        got, _ = tc.batch_ipv4(arena, sub, n, 0, want_flags=False)
    torch.cuda.synchronize()
    bad = int((_host(got) != _host(out)[idx]).sum())  # uint16 / uint32: no CUDA gather for them
    return {"segments": n, "mismatches": bad}


def check_devices(devices: list, backend: str):
    """None when every rank timed its own GPU, else the reason."""
    if backend != "nccl" or len(devices) < 2:
        return None
    keys = [d["pci"] or d["uuid"] for d in devices]
    if len(set(keys)) != len(keys):
        return f"ranks share a GPU: {keys}"
    return None


def launch_ranks(args) -> int:
    """`bench.py --gpus N` without a launcher: start N rank processes of this
    script (one per GPU, torchrun's environment, rendezvous on 127.0.0.1)
    before anything touches a GPU, and exit with their status.  N larger than
    the node's GPU count is refused (TCSUM_DIST_BACKEND=gloo rehearses more
    ranks than GPUs, ranks then sharing devices)."""
    from tcp_amd import dist as D
    backend = os.environ.get("TCSUM_DIST_BACKEND", "nccl")
    if not args.cpu_rehearsal:
        import torch
        ndev = torch.cuda.device_count()  # counts without initialising the GPU
        if args.gpus > ndev and backend == "nccl":
            print(f"bench.py: --gpus {args.gpus} but this node has {ndev} GPU(s); "
                  "refusing to time fewer GPUs than asked", file=sys.stderr)
            return 2
        from tcp_amd import build
        build.build()  # once, before the ranks start
    return D.spawn_ranks(args.gpus, [os.path.abspath(__file__)] + sys.argv[1:])


def rehearsal(args, rank, world) -> None:
    """The N>1 path on CPU: the same rank slices, barrier and max-over-ranks
    time as the GPU run, with a numpy byte sum over stand-in bytes in place of
    the kernel.  Prints a line marked "rehearsal"; never a measurement."""
    import numpy as np
    from tcp_amd import dist as D
    from tcp_amd import workload
    dist = D.init("gloo")
    b = workload.make_batch(args.config, rank=rank, n=4096)
    data = np.random.default_rng(b.byte_base).integers(0, 256, b.alloc_bytes, dtype=np.uint8)
    for _ in range(args.warmup):
        data.sum(dtype=np.uint64)
    D.barrier(dist)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        s = int(data.sum(dtype=np.uint64))
    dt = time.perf_counter() - t0
    D.barrier(dist)
    t = D.max_over_ranks(dist, dt)
    multi = rehearse_multi_device(b, data, world) if rank == 0 else None
    # the same post-timing checks as the GPU run: which device each rank used
    # (here: its CPU process) and the stand-in re-run against its timed result
    bad = int(int(data.astype(np.uint64).sum()) != s)
    dev = {"ordinal": None, "pci": None, "uuid": f"cpu-rank-{rank}-pid-{os.getpid()}", "name": "cpu (rehearsal)"}
    ranks = D.gather_objects(dist, {"rank": rank, "byte_base": int(b.byte_base), "packets": int(b.n),
                                    "payload_bytes": int(b.total_bytes), "stand_in_sum": s, "device": dev,
                                    "ms_per_step": dt * 1e3 / max(args.steps, 1),
                                    "self_check": {"segments": 1, "mismatches": bad}})
    wall = D.max_over_ranks(dist, time.perf_counter() - _T0)  # every rank: a collective
    if rank == 0:
        print(json.dumps({"rehearsal": "cpu-gloo (numpy stand-in for the kernel; not a measurement)",
                          "n_gpus": world, "steps": args.steps, "scaling": "weak",
                          "value": round(world * b.total_bytes * args.steps / t / GIB, 3),
                          "max_rank_s": t, "ranks": ranks, "devices": [r["device"] for r in ranks],
                          "ranks_ms_per_step": [round(r["ms_per_step"], 4) for r in ranks],
                          "ms_per_step_spread": {"min": round(min(r["ms_per_step"] for r in ranks), 4),
                                                 "max": round(max(r["ms_per_step"] for r in ranks), 4)},
                          "self_check": {"segments_per_rank": 1,
                                         "mismatches": sum(r["self_check"]["mismatches"] for r in ranks)},
                          "e2e": {"multi_device": multi},
                          "process_wall_s": round(wall, 2),
                          "driver_limit_s": DRIVER_LIMIT_S}),
              flush=True)
    D.barrier(dist)
    dist.destroy_process_group()


def rehearse_multi_device(b, data, ndev: int) -> dict:
    """e2e.multi_device's report on CPU: rank 0's batch cut into ndev shards
    by bytes (tcsum_host_batch_peso_multi's split, workload.shard_bounds), a
    numpy sum over each shard's bytes standing in for its device's host batch,
    reported through the same shard_report as the GPU child."""
    import numpy as np
    from tcp_amd import workload
    cut = workload.shard_bounds(b.descs["len"], ndev)
    shards = []
    for d in range(ndev):
        i0, i1 = int(cut[d]), int(cut[d + 1])
        lo = int(b.descs["offset"][i0]) if i1 > i0 else 0
        hi = int(b.descs["offset"][i1 - 1] + b.descs["len"][i1 - 1]) if i1 > i0 else 0
        t0 = time.perf_counter()
        data[lo:hi].sum(dtype=np.uint64)
        shards.append({"device": d, "rc": 0, "first": i0, "count": i1 - i0,
                       "bytes": int(b.descs["len"][i0:i1].sum()), "ms": (time.perf_counter() - t0) * 1e3})
    ident = lambda d: {"ordinal": d, "pci": None, "uuid": f"cpu-stand-in-{d}", "name": "cpu (rehearsal)"}  # noqa: E731
    return dict(shard_report(shards, ident), gpus=ndev, rehearsal=True)


def main():
    args = parse()
    KNOBS.extend(args.knob)
    if args.e2e_multi_child:
        e2e_multi_main(args.config)
        return
    from tcp_amd import dist as D
    if args.gpus > 1 and not D.launched() and not args.pmc_child:
        sys.exit(launch_ranks(args))
    rank, local, world = D.env()
    if world != max(args.gpus, 1):
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU "
              "(torchrun --nproc-per-node N ... --gpus N, or bench.py --gpus N alone)", file=sys.stderr)
        sys.exit(2)
    if args.cpu_rehearsal:
        rehearsal(args, rank, world)
        return
    n_gpus = max(world, 1)

    traffic, pmc_note, pmc_detail = None, "skipped", None
    trace, trace_note = None, "skipped"
    if not args.pmc_child and world == 1 and not args.no_pmc:
        traffic, pmc_note, pmc_detail = pmc_traffic(args.config)  # before this process touches the GPU
    if not args.pmc_child and world == 1 and not args.no_trace:
        trace, trace_note = rocprof_trace(args.config, args.steps, args.warmup, args.settle_ms)
    if not args.pmc_child and world == 1 and not (args.no_pmc and args.no_trace) and args.child_gap_ms > 0:
        time.sleep(args.child_gap_ms / 1e3)

    import torch
    from tcp_amd import build
    build.build()
    import tcp_amd as tc
    from tcp_amd import workload
    for kv in KNOBS:
        k, v = kv.split("=", 1)
        tc.debug_set(k, int(v))

    # one process per GPU; TCSUM_DIST_BACKEND=gloo rehearses N ranks on fewer
    # GPUs (ranks share devices round-robin; RCCL refuses two ranks per GPU)
    backend = os.environ.get("TCSUM_DIST_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    if ndev == 0 or (backend == "nccl" and local >= ndev):
        print(f"bench.py: rank {rank} (local {local}) has no GPU of its own ({ndev} on this node)",
              file=sys.stderr)
        sys.exit(2)
    dev = local % ndev
    torch.cuda.set_device(dev)
    dist = D.init(backend, dev)  # barrier + max-time only; no data-path collective

    global SETTLE_MS
    SETTLE_MS = 0.0 if args.pmc_child and not args.trace_child else max(0.0, args.settle_ms)
    if args.pmc_child:  # no probes: the tx probe launches k_tx_scatter, a step kernel by name
        r = time_config(torch, tc, workload, args.config, 0, args.steps, args.warmup, probes=False)
        # under rocprofv3: this process's own events, next to the trace's durations
        print(json.dumps({"child_ms_per_step": r["ms"] / args.steps, "child_launch_median_ms": r["launch_median_ms"]}),
              flush=True)
        return

    head = time_config(torch, tc, workload, args.config, rank, args.steps, args.warmup, dist, probes=False)
    ms = D.max_over_ranks(dist, head["ms"], device="cuda" if backend == "nccl" else "cpu")
    # after the timed region: every rank names its GPU and re-sums a sample of
    # its own slice against its timed results
    mine = {"rank": rank, "device": device_identity(torch, dev), "ms_per_step": head["ms"] / args.steps,
            "self_check": self_check(torch, tc, workload, head, 20240807 + rank)}
    ranks = D.gather_objects(dist, mine)
    devices = [dict(r["device"], rank=r["rank"]) for r in ranks]
    shared = check_devices(devices, backend)
    mism = sum(r["self_check"]["mismatches"] for r in ranks)
    run_probes(torch, tc, head)
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
        roof["traffic_raw"] = pmc_detail.pop("raw_bytes", None)
        roof["traffic_accounting"] = pmc_detail
    if trace is None:
        roof["rocprof_frac"] = None
        roof["rocprof_note"] = trace_note
    else:  # the same algorithmic bytes over the profiled child's median launch
        med_ns, mean_ns, nl, kname, step_ns, nk, child = trace
        roof["rocprof_frac"] = round(algorithmic_bytes(b) / (med_ns * 1e-9) / 1e9 / HBM_PEAK_GBS, 4)
        if nk > 1:  # the same bytes over every kernel of a step (their medians summed)
            roof["rocprof_step_frac"] = round(algorithmic_bytes(b) / (step_ns * 1e-9) / 1e9 / HBM_PEAK_GBS, 4)
        roof["rocprof"] = {"kernel": kname, "launches": nl, "median_us": round(med_ns / 1e3, 1),
                           "mean_us": round(mean_ns / 1e3, 1), "step_kernels": nk,
                           "step_median_us": round(step_ns / 1e3, 1),
                           "source": "rocprofv3 --kernel-trace --stats of bench.py --config "
                                     f"{args.config} (same K/W/settle), run as a child of this bench"}
        if child:
            # the traced child's own HIP events on the same launches: how much
            # the trace's per-dispatch durations exceed what the kernel takes
            # inside the traced process, and how much tracing slows it
            cl = child["child_launch_median_ms"] * 1e3
            roof["rocprof"]["child_events_launch_median_us"] = round(cl, 1)
            roof["rocprof"]["child_events_us_per_step"] = round(child["child_ms_per_step"] * 1e3, 1)
            roof["rocprof"]["trace_over_child_events"] = round(med_ns / 1e3 / cl, 4)
    # the line's frac: events over the K-launch window; per-launch event pairs
    # (untimed, the same K launches again) and the trace are reported beside
    # it, and frac_conservative is the lowest of the three
    if head.get("launch_median_ms"):
        roof["events_launch_median_us"] = round(head["launch_median_ms"] * 1e3, 1)
        roof["events_launch_frac"] = round(algorithmic_bytes(b) / (head["launch_median_ms"] * 1e-3) / 1e9
                                           / HBM_PEAK_GBS, 4)
    roof["frac_conservative"] = min(x for x in (roof["frac"], roof.get("events_launch_frac"),
                                                roof.get("rocprof_frac")) if x is not None)

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
        "devices": devices,
        **({"debug_knobs": KNOBS} if KNOBS else {}),
        # every rank's own time (the line's ms_per_step is their max): a
        # straggler GPU shows here on its own
        "ranks_ms_per_step": [round(r["ms_per_step"], 4) for r in ranks],
        "ms_per_step_spread": {"min": round(min(r["ms_per_step"] for r in ranks), 4),
                               "max": round(max(r["ms_per_step"] for r in ranks), 4),
                               "max_over_min": round(max(r["ms_per_step"] for r in ranks)
                                                     / max(1e-9, min(r["ms_per_step"] for r in ranks)), 4)},
        "self_check": {"segments_per_rank": mine["self_check"]["segments"], "mismatches": mism,
                       "what": "a seeded sample of each rank's segments re-summed in a separate launch after the "
                               "timed region, compared with the timed results (tx fill: filled again, must not "
                               "change a byte)"},
    }
    if shared or mism:
        if rank == 0:
            line["error"] = shared or f"{mism} sampled segments differ from the timed results"
            print(json.dumps(line), flush=True)
            print(f"bench.py: {line['error']}", file=sys.stderr)
        D.barrier(dist)
        sys.exit(2 if shared else 3)

    if world == 1:
        # the secondary configs first: timed after the host-memory legs below
        # (e2e, the drop-in calls) the 16-GiB configs[2] batch ran 3 % slower
        # than on its own (0.925 against 0.958 of spec, the same kernel's probe
        # rounds unaffected; profiles/r03/bench_tso_secondary_{plain,full}.json)
        extra = {}
        cfgs = [c for c in args.secondary.split(",") if c and c != args.config]
        pre, kept = {}, []
        if args.arena_policy == "prealloc":
            for cfg in cfgs:
                b2 = workload.make_batch(cfg)
                pre[cfg] = (b2,) + tuple(workload.materialize(b2))
            torch.cuda.synchronize()
        for i, cfg in enumerate(cfgs):
            if i and args.gap_ms > 0:
                time.sleep(args.gap_ms / 1e3)
            r = time_config(torch, tc, workload, cfg, 0, max(5, args.steps // 2), args.warmup, pre=pre.pop(cfg, None))
            extra[cfg] = result_entry(r, max(5, args.steps // 2))
            if cfg in ("tso", "mixed") and not args.no_cpu:  # CPU numbers for configs 2-4
                try:
                    extra[cfg]["cpu_baseline"] = cpu_baseline(torch, r, args.cpu_seconds / 2, args.cpu_kind,
                                                              cache_sample=False)
                except Exception as e:
                    extra[cfg]["cpu_baseline"] = {"value": None, "error": repr(e)}
            if args.arena_policy == "keep":
                kept.append((r["arena"], r["descs"]))
            del r
            if args.arena_policy == "free":
                torch.cuda.empty_cache()
        del kept
        torch.cuda.empty_cache()
        line["configs"] = extra
        line["secondary_arenas"] = {"policy": args.arena_policy, "gap_ms": args.gap_ms}
        if not args.no_cpu:
            try:
                line["cpu_baseline"] = cpu_baseline(torch, head, args.cpu_seconds, args.cpu_kind)
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

    # this rank's wall time from process start to the line: at N > 1 the
    # whole run (arena generation, timed steps, self-check; no secondary
    # configs, CPU or host-memory legs), which per-GPU work fixes whatever N
    wall = D.max_over_ranks(dist, time.perf_counter() - _T0, device="cuda" if backend == "nccl" else "cpu")
    line["process_wall_s"] = round(wall, 1)
    if world > 1:
        line["driver_limit_s"] = DRIVER_LIMIT_S
        line["wall_fraction_of_limit"] = round(wall / DRIVER_LIMIT_S, 3)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        D.barrier(dist)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
