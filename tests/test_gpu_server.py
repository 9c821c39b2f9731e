"""The queue server (tcsum_queue_server) on an MI355X: host-queue batches
served by a resident grid polling pinned memory give exactly the results of
the launch-per-batch path -- the reference's tx bytes, rx verdicts and both
checksums (tests/golden/ipv4_*.bin) -- over many back-to-back jobs, across the
grid leaving when idle and being relaunched, and with few workgroups (several
rounds per job)."""
from devcopy import down
import time

import numpy as np
import pytest

import golden_io as G

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def tc():
    import torch
    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    from tcp_amd import build
    build.build()
    import tcp_amd
    tcp_amd.plat_init(0)
    return tcp_amd


@pytest.fixture
def server(tc, dbg):
    def start(wgs=64, idle_ms=10):
        dbg(server_wgs=str(wgs))
        dbg(server_idle_ms=str(idle_ms))
        tc.queue_server(True)
    yield start
    tc.queue_server(False)


def host_copy(tc, data: np.ndarray, where: str, shift: int = 0):
    n = data.size + shift + 64
    if where == "pinned":
        ha = tc.HostArena(n)
        ha.array[:] = 0
        view = ha.array[shift:]
        view[: data.size] = data
        return (ha if shift == 0 else view), view, ha
    view = np.zeros(n, np.uint8)[shift:]
    view[: data.size] = data
    return view, view, None


@pytest.mark.parametrize("wgs", [1, 5, 64])
@pytest.mark.parametrize("where,shift", [("pinned", 0), ("pinned", 3), ("pageable", 1)])
def test_server_golden(tc, oracle, server, wgs, where, shift):
    server(wgs=wgs)
    # sums
    cases, pool = G.ipv4_cases()
    arg, view, keep = host_copy(tc, pool, where, shift)
    for _ in range(3):
        out, flags = tc.host_batch_ipv4(arg, G.pkt_descs(cases, tc.PKT_DTYPE))
        np.testing.assert_array_equal(out & 0xFFFF, cases["ip"])
        np.testing.assert_array_equal(out >> 16, cases["l4"])
        np.testing.assert_array_equal(flags, cases["flags"])
    # tx fill in place
    cases, pin, pout = G.ipv4_tx_cases()
    arg, view, keep = host_copy(tc, pin, where, shift)
    view[pin.size:] = 0xA5
    flags = tc.host_batch_ipv4_tx_fill(arg, G.pkt_descs(cases, tc.PKT_DTYPE))
    np.testing.assert_array_equal(view[: pout.size], pout)
    assert (view[pin.size:] == 0xA5).all()
    np.testing.assert_array_equal(flags, cases["flags"])
    # rx verdicts
    cases, pool = G.ipv4_rx_cases()
    arg, view, keep = host_copy(tc, pool, where, shift)
    pk = G.pkt_descs(cases, tc.PKT_DTYPE)
    verdict, out, flags = tc.host_batch_ipv4_rx_verify(arg, pk)
    np.testing.assert_array_equal(verdict, cases["verdict"])
    np.testing.assert_array_equal(flags, cases["flags"])
    exp, _ = oracle.batch_ipv4(pool, pk)
    np.testing.assert_array_equal(out, exp)


def test_server_many_small_queues(tc, oracle, server):
    """500 back-to-back netif-queue-sized jobs (1..50 frames, random subsets of
    a 4,096-frame pinned pool, rx and sums interleaved): every job's answer
    equals the oracle's for exactly its frames -- no job sees another's
    descriptors or results."""
    server(wgs=16)
    from tcp_amd import workload
    b = workload.make_batch("mixed_rx", n=4096)
    arena, _ = workload.materialize(b)
    ha = tc.HostArena(arena.numel())
    ha.array[:] = down(arena)
    want_out, want_flags = oracle.batch_ipv4(ha.array, b.descs)
    want_v, _ = oracle.batch_ipv4_rx_verify(ha.array, b.descs)
    rng = np.random.default_rng(11)
    for j in range(500):
        idx = rng.choice(b.n, size=int(rng.integers(1, 51)), replace=False)
        pk = b.descs[idx]
        if j % 2:
            out, flags = tc.host_batch_ipv4(ha, pk)
            np.testing.assert_array_equal(out, want_out[idx])
            np.testing.assert_array_equal(flags, want_flags[idx])
        else:
            verdict, out, _ = tc.host_batch_ipv4_rx_verify(ha, pk)
            np.testing.assert_array_equal(verdict, want_v[idx])
            np.testing.assert_array_equal(out, want_out[idx])
    ha.free()


def test_server_idles_out_and_relaunches(tc, oracle, server):
    """A 2 ms idle limit: the grid leaves between jobs spaced 20 ms apart and
    the next call relaunches it; device-wide syncs complete meanwhile."""
    import torch
    server(wgs=8, idle_ms=2)
    cases, pool = G.ipv4_cases()
    arg, view, keep = host_copy(tc, pool, "pinned")
    pk = G.pkt_descs(cases, tc.PKT_DTYPE)
    for _ in range(5):
        out, _ = tc.host_batch_ipv4(arg, pk)
        np.testing.assert_array_equal(out & 0xFFFF, cases["ip"])
        time.sleep(0.02)
        torch.cuda.synchronize()  # returns once the idle grid has left


def test_server_off_restores_launch_path(tc, server):
    server(wgs=4)
    cases, pool = G.ipv4_cases()
    arg, view, keep = host_copy(tc, pool, "pinned")
    pk = G.pkt_descs(cases, tc.PKT_DTYPE)
    a, _ = tc.host_batch_ipv4(arg, pk)
    tc.queue_server(False)
    b, _ = tc.host_batch_ipv4(arg, pk)
    np.testing.assert_array_equal(a, b)
