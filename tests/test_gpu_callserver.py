"""The call server (tcsum_call_server) on an MI355X: the three synchronous
drop-in symbols served by one resident wave give the reference's results and
side effects on every golden case, survive the wave idling out, hand long
ranges to the launch path, and serve the reference's own objects linked
against libtcsum.so (TCSUM_CALL_SERVER=1, no code change)."""
import os
import time

import numpy as np
import pytest

import golden_io as G
import test_gpu_parity as P

pytestmark = pytest.mark.gpu

torch = P.torch
tc = P.tc


@pytest.fixture
def served(tc, dbg):
    dbg(server_idle_ms="50")
    tc.call_server(True)
    yield
    tc.call_server(False)


def test_served_kats(tc, served):
    P.test_kats(tc)


def test_served_checksum16_golden(tc, served):
    P.test_checksum16_golden(tc)


def test_served_pktbuf_checksum16_golden(tc, served):
    P.test_pktbuf_checksum16_golden(tc)


def test_served_checksum_peso_golden(tc, served):
    P.test_checksum_peso_golden(tc)


def test_served_idle_out_and_relaunch(tc, dbg):
    """The wave leaves after 2 ms without a call; the next call relaunches it."""
    dbg(server_idle_ms="2")
    tc.call_server(True)
    try:
        hdr = bytes.fromhex("450000730000400040110000c0a80001c0a800c7")
        for _ in range(5):
            assert tc.checksum16(0, hdr, 20, 0, 1) == 0x61B8
            time.sleep(0.02)  # 10x the idle limit: the wave has left
            assert tc.checksum16(1, hdr, 20, 0, 0) == tc.checksum16(1, hdr, 20, 0, 0)
    finally:
        tc.call_server(False)


def test_served_long_range_takes_launch_path(tc, served, oracle):
    """A pktbuf range over 64 KiB (the served staging) is summed by a launch,
    between served calls, with the same result as the oracle."""
    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, 200_000, dtype=np.uint8).tobytes()
    pieces = [data[i: i + 127] for i in range(0, len(data), 127)]
    for n in (65536, 65537, 200_000):  # the last served size, then launches
        buf = tc.PktBuf(pieces)
        got = tc.pktbuf_checksum16(buf, n, 0x1234, 1)
        assert got == oracle.pieces_checksum16(pieces, n, 0x1234, 1), n
        assert buf.cursor()[0] == n
        # a served call right after the launch path
        assert tc.checksum16(1, data[:1500], 1500, 7, 1) == oracle.checksum16(1, data[:1500], 1500, 7, 1)


def test_served_reference_objects(tc):
    """oracle/_ref/dropin_stack with TCSUM_CALL_SERVER=1: the reference's own
    pktbuf/tools objects, every pktbuf/peso golden case through the wave."""
    import subprocess
    exe = os.path.join(os.path.dirname(G.GOLDEN), "..", "oracle", "_ref", "dropin_stack")
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref not built (needs /root/reference at build time)")
    env = dict(os.environ, TCSUM_CALL_SERVER="1")
    r = subprocess.run([exe, G.GOLDEN], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "2749/2749" in r.stdout
