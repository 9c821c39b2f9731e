"""integration/net_checksum_gpu.patch: the stack's call sites as a compiled
artifact.  CPU: the patch applies to a copy of the reference, the patched
stack compiles with and without NET_CHECKSUM_GPU and links against
libtcsum.so with no unresolved checksum symbol, and configs[0] (UDP + TCP
echo over the loop netif) runs on the reference's own CPU checksum.  GPU: the
same echo with every checksum filled and tested through the GPU batches."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INTEG = os.path.join(ROOT, "integration")
BUILD = os.path.join(INTEG, "_build")
HAVE_REF = os.path.isdir("/root/reference/net/src")


@pytest.mark.skipif(not HAVE_REF, reason="needs /root/reference (build container)")
@pytest.mark.timeout(300)
def test_patch_applies_and_links():
    r = subprocess.run(["make", "-C", INTEG, "all"], capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "integration check: patch applies, GPU and CPU builds link" in r.stdout


@pytest.mark.skipif(not HAVE_REF, reason="needs /root/reference (build container)")
@pytest.mark.timeout(200)
def test_loop_echo_cpu_reference():
    """configs[0] as the reference runs it (its CPU checksum), over loopback."""
    exe = os.path.join(BUILD, "loop_echo_cpu")
    subprocess.run(["make", "-C", INTEG, exe], check=True, capture_output=True, timeout=280)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "udp: 200 datagrams" in r.stdout and "tcp: 65536 bytes echoed intact" in r.stdout


def _batch_hist(out: str):
    """loop_echo's tx batch-size histogram: counts of 1, 2-3, 4-7, ... frames."""
    line = next(ln for ln in out.splitlines() if ln.startswith("batch sizes"))
    tx = line.split("tx [", 1)[1].split("]", 1)[0]
    return [int(part.split()[-1]) for part in tx.split("|")]


@pytest.mark.skipif(not HAVE_REF, reason="needs /root/reference (build container)")
@pytest.mark.timeout(300)
def test_loop_echo_coalescing_cpu_double():
    """configs[0] through the patched stack's own glue (net_csum_gpu.c: frames
    held until the work thread is idle, one fill per flush) with the oracle
    behind the engine's entry points: 1 MiB over TCP echoed intact, no
    retransmission stall, and batches of more than one frame; with
    NET_CSUM_COALESCE=0 every batch is one frame, as in round 3."""
    exe = os.path.join(BUILD, "loop_echo_dbl")
    subprocess.run(["make", "-C", INTEG, exe], check=True, capture_output=True, timeout=280)
    for _ in range(3):
        r = subprocess.run([exe, "--rounds", "100", "--tcp-bytes", "1048576"], capture_output=True, text=True,
                           timeout=90)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        assert "tcp: 1048576 bytes echoed intact" in r.stdout
        assert "tcp rexmit" not in r.stdout + r.stderr
        h = _batch_hist(r.stdout)
        assert sum(h[1:]) > 0, h  # frames did leave together
    r = subprocess.run([exe, "--rounds", "100", "--tcp-bytes", "262144"], capture_output=True, text=True,
                       timeout=90, env=dict(os.environ, NET_CSUM_COALESCE="0"))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    h = _batch_hist(r.stdout)
    assert h[0] > 0 and sum(h[1:]) == 0, h


@pytest.mark.gpu
@pytest.mark.timeout(200)
def test_loop_echo_gpu():
    """configs[0] on the patched stack: tx checksums filled by the batched
    fill in loop_xmit, rx checksums from the batched sums in do_netif_in."""
    exe = os.path.join(BUILD, "loop_echo")
    assert os.path.exists(exe), "built in the build container by make -C integration (__graft_entry__.build)"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=90)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "udp: 200 datagrams" in r.stdout and "tcp: 65536 bytes echoed intact" in r.stdout
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("engine:")][0]
    print(line)


# ---------------------------------------------------------------- pcap driver
# integration/pcap_wire.c: the reference's plat/netif_pcap.c (patched) run for
# real over the libpcap test double: tx fixtures out through xmit_thread's
# batched fill + pcap_inject, rx fixtures in through recv_thread + the batched
# do_netif_in, forced engine / inject failures, and the loop netif's fill
# concurrently with the pcap xmit_thread's.
GOLDEN = os.path.join(ROOT, "tests", "golden")
PHASES = ("tx", "rx", "rx_replies", "fault_tx", "fault_rx", "fault_inject", "concurrent")


def _phases(out: str) -> dict:
    got = {}
    for ln in out.splitlines():
        if ln.startswith("phase "):
            name, rest = ln[len("phase "):].split(": ", 1)
            got[name] = rest
    return got


def _run_pcap_wire(exe: str, timeout: int, env=None, stderr_out=None) -> str:
    r = subprocess.run([exe, GOLDEN], capture_output=True, text=True, timeout=timeout, env=env)
    if stderr_out is not None:
        stderr_out.append(r.stderr)
    ph = _phases(r.stdout)
    summary = "\n".join(f"{k}: {v}" for k, v in ph.items())
    assert r.returncode == 0, summary + "\n" + r.stdout[-3000:] + r.stderr[-3000:]
    for p in PHASES:
        assert ph.get(p, "").startswith("ok"), f"phase {p}: {ph.get(p)}\n{summary}"
    # every fixture went through (tx: all 1,481 frames; rx: every non-fragment
    # frame that fits the Ethernet MTU and has defined reference behaviour)
    assert ph["tx"].startswith("ok 1481 frames"), ph["tx"]
    n_rx = int(ph["rx"].split()[1])
    assert n_rx > 1900, ph["rx"]
    # the failures were logged where the stack logs errors
    assert "batched checksum fill failed on the device" in r.stdout
    assert "summing them one by one" in r.stdout
    assert "pcap send failed" in r.stdout
    print(summary)
    return r.stdout


@pytest.mark.skipif(not HAVE_REF, reason="needs /root/reference (build container)")
@pytest.mark.timeout(300)
def test_pcap_driver_cpu_double():
    """The patched pcap driver end to end with the oracle behind the engine's
    entry points (integration/tcsum_cpu_double.c): the stack-side logic."""
    exe = os.path.join(BUILD, "pcap_wire_cpu")
    # always: make's own dependencies skip the work when nothing changed, and
    # an edit to pcap_wire.c or either patch is never tested on a stale binary
    subprocess.run(["make", "-C", INTEG, exe], check=True, capture_output=True,
                   timeout=280)
    _run_pcap_wire(exe, 240)


@pytest.mark.skipif(not HAVE_REF, reason="needs /root/reference (build container)")
@pytest.mark.timeout(600)
def test_pcap_driver_threadsanitizer():
    """Every thread of the patched stack (work_thread's loop_xmit fill and rx
    batches, the pcap recv_thread / xmit_thread) under ThreadSanitizer, three
    runs: no data race is reported (TSan exits 66 when it finds one).  The
    stack is built with the one-line fix for the reference's own ICMP
    header overflow (integration/ref_icmp_fix.patch),
    which TSan otherwise reports as a race on the block it overruns."""
    r = subprocess.run(["make", "-C", INTEG, "tsan"], capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    exe = os.path.join(BUILD, "pcap_wire_tsan")
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=0 exitcode=66")
    for _ in range(3):
        err = []
        out = _run_pcap_wire(exe, 180, env=env, stderr_out=err)  # rc 66 on a report fails inside
        # TSan writes its reports to stderr
        assert "WARNING: ThreadSanitizer" not in err[0] and "WARNING: ThreadSanitizer" not in out


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_pcap_driver_gpu():
    """The patched plat/netif_pcap.c with libtcsum.so: every frame xmit_thread
    injects carries the checksums the reference stack stored (stack_tx_out),
    every received frame's verdict equals the reference stack's, the stack's
    own replies are filled exactly as the oracle fills them, and engine
    failures are logged, counted and handled."""
    exe = os.path.join(BUILD, "pcap_wire")
    assert os.path.exists(exe), "built in the build container by make -C integration (__graft_entry__.build)"
    out = _run_pcap_wire(exe, 240)
    eng = [ln for ln in out.splitlines() if ln.startswith("engine final")]
    print(eng[-1] if eng else "")
