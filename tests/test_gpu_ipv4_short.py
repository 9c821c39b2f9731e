"""Short IPv4 packets on the narrow lane groups the router gives them
(csum_launch.h ipv4_short_shape: 2 x 4 under ~96 B (rx ~128 B), 4 x 4 under ~250 B, 8 x 4 / 8 x 6 / 8 x 3
to ~1.3 KiB, 16 x 4 / 16 x 3 / 16 x 6 to ~4 KiB; rx keeps 16+ lanes past
~1.3 KiB).  Fuzzed packets around each mean (headers mostly plausible, some
short frames, random arena phase) through sums, rx verify, tx offload and
both tx fill forms, against the oracle (net/src/tools.c:24-75, ipv4.c,
tcp_in.c / udp.c for the verdicts).  Also each narrow shape forced through
the debug knobs on the reference's own packets (tests/golden)."""
from devcopy import down, up
import golden_io as G
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available(), "gpu tests need an MI355X"
    return t


@pytest.fixture(scope="module")
def tc(torch):
    from tcp_amd import build
    build.build()
    import tcp_amd
    tcp_amd.plat_init(0)
    return tcp_amd


MEANS = [40, 64, 100, 200, 300, 600, 1000, 1500, 2000, 3000]


@pytest.mark.parametrize("mean", MEANS)
def test_routed_short_shapes_match_the_oracle(tc, torch, oracle, mean):
    from test_gpu_flat import _arena, _headers, _pk, _stream
    rng = np.random.default_rng(4000 + mean)
    n = int(min(6000, (12 << 20) // mean))
    lens = rng.integers(max(1, mean // 2), mean * 3 // 2 + 1, n).astype(np.int64)
    short = rng.random(n) < 0.05
    lens[short] = rng.integers(0, 20, int(short.sum()))
    offs = _stream(lens, int(rng.integers(0, 64)))
    host = _arena(rng, int(offs[-1] + lens[-1]) + 256)
    _headers(rng, host, offs, lens, valid=0.9)
    pk = _pk(tc, offs, lens)
    total = int(lens.sum())
    arena = up(torch.from_numpy(host))
    d = tc.descs_to_device(pk)
    exp, efl = oracle.batch_ipv4(host, pk, nthreads=8)
    out, fl = tc.batch_ipv4(arena, d, n, total)
    np.testing.assert_array_equal(down(out), exp)
    np.testing.assert_array_equal(down(fl), efl)
    ev, evfl = oracle.batch_ipv4_rx_verify(host, pk, nthreads=8)
    v, vfl = tc.batch_ipv4_rx_verify(arena, d, n, total)
    np.testing.assert_array_equal(down(v), ev)
    np.testing.assert_array_equal(down(vfl), evfl)
    want = host.copy()
    oracle.batch_ipv4_tx_fill(want, pk, nthreads=8)
    tout, tfl = tc.batch_ipv4_tx_offload(arena, d, n, total)
    applied = host.copy()
    tc.tx_apply_batch(applied, pk, down(tout), down(tfl))
    np.testing.assert_array_equal(applied, want)
    for split in (0, 1):
        a2 = up(torch.from_numpy(host.copy()))
        with tc.debug(tx_split=split):
            tc.batch_ipv4_tx_fill(a2, d, n, total)
        np.testing.assert_array_equal(down(a2)[: host.size], want)


def _dev(torch, a):
    return up(torch.from_numpy(np.concatenate([a, np.zeros(64, np.uint8)])))


@pytest.mark.parametrize("g,u", [(2, 4), (4, 4), (8, 3), (8, 4), (8, 6)])
def test_forced_narrow_shapes_on_golden_packets(tc, torch, g, u):
    cases, ipool = G.ipv4_cases()
    pk = G.pkt_descs(cases, tc.PKT_DTYPE)
    rcases, rpool = G.ipv4_rx_cases()
    rpk = G.pkt_descs(rcases, tc.PKT_DTYPE)
    tcases, pin, pout = G.ipv4_tx_cases()
    tpk = G.pkt_descs(tcases, tc.PKT_DTYPE)
    with tc.debug(lanes=g, loads=u):
        out, flags = tc.batch_ipv4(_dev(torch, ipool), tc.descs_to_device(pk), pk.size)
        out = down(out)
        np.testing.assert_array_equal(out & 0xFFFF, cases["ip"])
        np.testing.assert_array_equal(out >> 16, cases["l4"])
        np.testing.assert_array_equal(down(flags), cases["flags"])
        verdict, vfl = tc.batch_ipv4_rx_verify(_dev(torch, rpool), tc.descs_to_device(rpk), rpk.size)
        np.testing.assert_array_equal(down(verdict), rcases["verdict"])
        np.testing.assert_array_equal(down(vfl), rcases["flags"])
        for split in (0, 1):
            with tc.debug(tx_split=split):
                arena = _dev(torch, pin)
                tc.batch_ipv4_tx_fill(arena, tc.descs_to_device(tpk), tpk.size)
                np.testing.assert_array_equal(down(arena)[: pout.size], pout)
