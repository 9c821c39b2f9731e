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
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", INTEG, "all"], check=True, capture_output=True, timeout=280)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "udp: 200 datagrams" in r.stdout and "tcp: 65536 bytes echoed intact" in r.stdout


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
