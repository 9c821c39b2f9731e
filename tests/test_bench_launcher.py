"""bench.py's N-rank launcher on CPU (gloo): `bench.py --gpus N` with no
launcher starts N ranks itself; a GPU count the node cannot provide, or a
WORLD_SIZE that differs from --gpus, fails loudly."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def run(args, env=None, timeout=240):
    e = dict(os.environ)
    for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=timeout,
                          env=e, cwd=ROOT)


@pytest.mark.timeout(300)
def test_launcher_world2_rehearsal():
    r = run(["--gpus", "2", "--cpu-rehearsal", "--steps", "3", "--warmup", "1"])
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1  # rank 0 alone prints
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["scaling"] == "weak" and line["value"] > 0
    ranks = sorted(line["ranks"], key=lambda x: x["rank"])
    assert [x["rank"] for x in ranks] == [0, 1]
    # weak scaling: consecutive, disjoint slices of one global stream
    assert ranks[0]["byte_base"] == 0 and ranks[1]["byte_base"] >= ranks[0]["payload_bytes"]
    assert ranks[0]["stand_in_sum"] != ranks[1]["stand_in_sum"]
    # each rank names the device it timed; rank 0's line lists them all
    devs = line["devices"]
    assert len(devs) == 2 and len({d["uuid"] for d in devs}) == 2
    # each rank re-ran its stand-in after the timed region: no mismatch
    assert line["self_check"]["mismatches"] == 0 and line["self_check"]["segments_per_rank"] >= 1
    # every rank's own time, so a straggler shows by itself
    assert len(line["ranks_ms_per_step"]) == 2 and all(t > 0 for t in line["ranks_ms_per_step"])
    sp = line["ms_per_step_spread"]
    assert sp["min"] == min(line["ranks_ms_per_step"]) and sp["max"] == max(line["ranks_ms_per_step"])
    check_multi_device(line, 2)


def check_multi_device(line, world):
    """e2e.multi_device names every shard's device and times it on its own
    (VERDICT r04 item 7), the way the device-resident line names ranks."""
    m = line["e2e"]["multi_device"]
    assert m["gpus"] == world and len(m["shards"]) == world == len(m["devices"])
    assert [s["device"]["ordinal"] for s in m["shards"]] == list(range(world))
    assert all(set(s["device"]) >= {"ordinal", "pci", "uuid", "name"} for s in m["shards"])
    assert all(s["ms"] > 0 and s["gib_s"] > 0 and s["rc"] == 0 for s in m["shards"])
    assert sum(s["packets"] for s in m["shards"]) == line["ranks"][0]["packets"]
    sp = m["shard_ms_spread"]
    assert sp["max"] >= sp["min"] > 0 and sp["max_over_min"] >= 1.0


def test_shared_gpu_is_refused():
    """Under RCCL two ranks on one GPU make the aggregate meaningless: the
    bench's device check names them (bench.py exits 2 on it)."""
    sys.path.insert(0, ROOT)
    import bench
    a = {"ordinal": 0, "pci": "0000:05:00", "uuid": "u0"}
    b = {"ordinal": 1, "pci": "0000:15:00", "uuid": "u1"}
    assert bench.check_devices([a, b], "nccl") is None
    assert "share a GPU" in bench.check_devices([a, dict(a)], "nccl")
    assert bench.check_devices([a, dict(a)], "gloo") is None  # a rehearsal may share on purpose


@pytest.mark.timeout(300)
def test_launcher_refuses_missing_gpus():
    """No GPU here: --gpus 2 must exit nonzero, not time fewer GPUs."""
    r = run(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert r.returncode != 0
    assert "GPU" in r.stderr


@pytest.mark.timeout(120)
def test_world_size_must_match_gpus():
    r = run(["--gpus", "2", "--steps", "1"], env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr
    r = run(["--steps", "1", "--cpu-rehearsal"], env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2


@pytest.mark.timeout(120)
def test_spawn_ranks_failing_rank_ends_the_others(tmp_path):
    """A rank that fails while rank 0 is still running (e.g. waiting in a
    barrier) ends the whole launch at once with its exit status."""
    import time
    sys.path.insert(0, ROOT)
    from tcp_amd import dist as D
    prog = tmp_path / "rank.py"
    prog.write_text("import os, sys, time\n"
                    "if os.environ['RANK'] == '1':\n"
                    "    sys.exit(3)\n"
                    "time.sleep(60)\n")
    t0 = time.monotonic()
    assert D.spawn_ranks(2, [str(prog)]) == 3
    assert time.monotonic() - t0 < 30
    assert D.spawn_ranks(2, [str(prog)], extra_env={"RANK": "0"}, timeout=1.0) == 124  # both sleep: time-out


def test_calibrated_traffic_accounting():
    """bench.py's per-class counter accounting: raw counters equal to what the
    classes report on their own give exactly the classes' bytes; 5 % more
    FETCH_SIZE gives 5 % more read traffic; every class a config uses has a
    calibration entry."""
    sys.path.insert(0, ROOT)
    import bench
    from tcp_amd import workload
    for cfg in ("mtu", "tso", "mixed", "mixed_tx", "mixed_rx", "mixed_txo"):
        cls = bench.access_classes(workload.make_batch(cfg, n=4096))
        assert all(k in bench.PMC_CALIB for k, _ in cls)
        exp = {c: sum(b * bench.PMC_CALIB[k] for (k, cc), b in cls.items() if cc == c)
               for c in ("FETCH_SIZE", "WRITE_SIZE")}
        nominal = sum(cls.values())
        t, detail = bench.calibrated_traffic(cls, exp)
        assert abs(t - nominal) < 1e-6 * nominal
        t5, _ = bench.calibrated_traffic(cls, dict(exp, FETCH_SIZE=exp["FETCH_SIZE"] * 1.05))
        reads = sum(b for (k, c), b in cls.items() if c == "FETCH_SIZE")
        assert abs(t5 - nominal - 0.05 * reads) < 1e-6 * nominal


def test_raw_traffic_shows_write_amplification():
    """traffic_raw: the guide's corrections only, each
    counter over the algorithmic bytes of its direction.  Counters as round
    4's mixed_tx line read them (FETCH x2 ~ algorithmic reads, 65.96 MB of
    writes) give WRITE ~5.2x the 12 B per packet the deferred fill stores,
    ~15.7x the 4 B of checksum fields, and total ~1.02x;
    the headline's descriptors fetched twice show as FETCH ~1.016x."""
    sys.path.insert(0, ROOT)
    import bench
    from tcp_amd import workload
    tx = workload.make_batch("mixed_tx")
    rd, wr = bench.algorithmic_split(tx)
    assert wr == 4 * tx.n and rd + wr == bench.algorithmic_bytes(tx)
    r = bench.raw_traffic(tx, {"FETCH_SIZE": rd / 2 * 1.0004, "WRITE_SIZE": 65.96e6})
    assert 5.0 < r["write_vs_step_stores"] < 5.4  # over the 12 B the deferred fill stores per packet
    assert 15.0 < r["write_vs_algorithmic_write"] < 16.5  # over the 4 B of checksum fields
    assert 1.01 < r["total_vs_algorithmic"] < 1.03
    mtu = workload.make_batch("mtu")
    rd, wr = bench.algorithmic_split(mtu)
    r = bench.raw_traffic(mtu, {"FETCH_SIZE": (rd + 24 * mtu.n) / 2, "WRITE_SIZE": wr})
    assert abs(r["fetch_vs_algorithmic_read"] - 1.0 - 24 * mtu.n / rd) < 1e-3
    assert r["write_vs_algorithmic_write"] == 1.0


def test_step_counter_counts_only_kernels_of_every_step(tmp_path):
    """A step's counter value: the median launch of each kernel the step runs,
    summed (the deferred tx fill's two kernels); a setup kernel launched once
    (rx's preparing tx fill, the synthetic fill) is no part of it -- round 4's
    rx line first counted it and reported 2x its traffic."""
    sys.path.insert(0, ROOT)
    import bench

    def csv_of(rows):
        f = tmp_path / f"c{len(list(tmp_path.iterdir()))}.csv"
        f.write_text("Kernel_Name,Counter_Name,Counter_Value\n" +
                     "".join(f'"{k}(args)",FETCH_SIZE,{v}\n' for k, v in rows))
        return str(f)

    rx = [("void tcsum::k_ipv4<32, 6, 1, 256, 0>", 200.0), ("tcsum::k_tx_scatter", 50.0),
          ("tcsum::k_synth_fill", 999.0)] + [("void tcsum::k_ipv4<16, 6, 2, 256, 0>", 100.0 + i) for i in range(7)]
    assert bench.step_counter([csv_of(rx)], "FETCH_SIZE") == 103.0
    tx = [("void tcsum::k_ipv4<32, 6, 1, 256, 0>", 100.0)] * 7 + [("tcsum::k_tx_scatter", 10.0)] * 7
    assert bench.step_counter([csv_of(tx)], "FETCH_SIZE") == 110.0
    assert bench.step_counter([csv_of([("tcsum::k_synth_fill", 1.0)])], "FETCH_SIZE") is None


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [4, 8])
def test_launcher_rehearsal_many_ranks(world):
    """configs[4]'s layout (8 ranks, one per GPU) rehearsed on CPU: every rank
    times its own consecutive slice of the one global stream, rank 0 alone
    prints, the devices are distinct and every self-check is clean."""
    r = run(["--gpus", str(world), "--cpu-rehearsal", "--steps", "2", "--warmup", "1"], timeout=280)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert line["n_gpus"] == world and len(line["devices"]) == world
    assert len({d["uuid"] for d in line["devices"]}) == world
    ranks = sorted(line["ranks"], key=lambda x: x["rank"])
    assert [x["rank"] for x in ranks] == list(range(world))
    for a, b in zip(ranks, ranks[1:]):
        assert b["byte_base"] >= a["byte_base"] + a["payload_bytes"]
    assert line["self_check"]["mismatches"] == 0
    assert len(line["ranks_ms_per_step"]) == world and line["ms_per_step_spread"]["max"] >= \
        line["ms_per_step_spread"]["min"] > 0
    # the slowest rank's wall time from process start is in the line, and the
    # whole N-rank run fits the driver's limit with margin
    assert 0 < line["process_wall_s"] < 0.5 * line["driver_limit_s"]
    check_multi_device(line, world)


def test_cpu_allowance_reads_cgroup_limits(tmp_path):
    """The all-core CPU baseline runs as many threads as the process may use:
    the affinity mask, and the tightest cgroup cpuset and CPU quota on the
    way to the root (v2 cpu.max / cpuset.cpus.effective; v1 cfs quota and
    cpuset), not the host's os.cpu_count()."""
    import os

    import bench
    assert bench._cpuset_count("0-15,32-47\n") == 32 and bench._cpuset_count("3") == 1
    aff = len(os.sched_getaffinity(0))
    # v2: a 16-CPU quota on the lease's cgroup, 32 CPUs in its parent's cpuset
    root = tmp_path / "v2"
    (root / "lease" / "job").mkdir(parents=True)
    (root / "lease" / "cpu.max").write_text("1600000 100000\n")
    (root / "cpuset.cpus.effective").write_text("0-15,32-47\n")
    (root / "lease" / "job" / "cpu.max").write_text("max 100000\n")
    (tmp_path / "cg2").write_text("0::/lease/job\n")
    a = bench.cpu_allowance(str(root), str(tmp_path / "cg2"))
    assert a["cpu_quota"] == 16.0 and a["cpuset"] == 32 and a["effective"] == min(aff, 16)
    # v1: cfs quota of 2.5 CPUs under the cpu controller's path
    root = tmp_path / "v1"
    (root / "cpu" / "grp").mkdir(parents=True)
    (root / "cpu" / "grp" / "cpu.cfs_quota_us").write_text("250000\n")
    (root / "cpu" / "grp" / "cpu.cfs_period_us").write_text("100000\n")
    (tmp_path / "cg1").write_text("4:cpu,cpuacct:/grp\n3:cpuset:/\n")
    a = bench.cpu_allowance(str(root), str(tmp_path / "cg1"))
    assert a["cpu_quota"] == 2.5 and a["effective"] == min(aff, 2)
    # nothing limits: the affinity mask
    (tmp_path / "cg0").write_text("0::/\n")
    a = bench.cpu_allowance(str(tmp_path / "empty"), str(tmp_path / "cg0"))
    assert "cpu_quota" not in a and a["effective"] == aff
