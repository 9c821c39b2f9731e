"""The deferred tx fill's warming loads (k_tx_scatter<true>, debug knob
"tx_warm"): before its 2-B stores each lane loads the dword
under each of its packet's fields.  The loads may not change a stored byte or
leave the packet's own dwords: fuzzed packets of 0..9000 B (many of them
20..60-B TCP / UDP / ICMP frames whose L4 field sits at the frame's end), at
every arena phase, the last frame ending at the end of its allocation,
warm and cold, against the oracle's tx fill (net/src/ipv4.c:643,656,
tcp_out.c:19-20, udp.c:320-321, icmpv4.c:45-58).  The same fill on a
pinned host arena (the kernel reads and writes host memory in place; the
library picks the plain stores there, as hipPointerGetAttributes calls it
host memory) gives the same bytes."""
from devcopy import down
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


def _batch(tc, seed, phase):
    from test_gpu_flat import _arena, _headers, _pk, _stream
    rng = np.random.default_rng(900 + seed)
    n = 3000
    kind = rng.integers(0, 3, n)
    lens = np.where(kind == 0, rng.integers(20, 61, n),
                    np.where(kind == 1, rng.integers(0, 20, n), rng.integers(20, 9001, n))).astype(np.int64)
    lens[-1] = 28  # a UDP header and nothing more, last in the arena
    offs = _stream(lens, phase)
    host = _arena(rng, int(offs[-1] + lens[-1]))  # no byte after the last frame
    _headers(rng, host, offs, lens, valid=0.95)
    o = int(offs[-1])
    host[o] = 0x45
    host[o + 2: o + 4] = [0, 28]
    host[o + 6: o + 8] = 0
    host[o + 9] = 17
    return host, _pk(tc, offs, lens)


def _exact(torch, host):
    """The bytes in a device allocation of exactly their size."""
    t = torch.empty(host.size, dtype=torch.uint8, device="cuda")
    t.copy_(torch.from_numpy(host.copy()).pin_memory())
    return t


@pytest.mark.parametrize("phase", [0, 1, 2, 3, 5, 13])
@pytest.mark.parametrize("seed", range(2))
def test_warm_scatter_matches_oracle(tc, torch, oracle, seed, phase):
    host, pk = _batch(tc, seed, phase)
    want = host.copy()
    oracle.batch_ipv4_tx_fill(want, pk, nthreads=8)
    assert (want != host).any()
    d = tc.descs_to_device(pk)
    total = int(pk["len"].sum())
    for warm in (None, 0):
        arena = _exact(torch, host)
        with tc.debug(tx_split=1, tx_warm=warm):
            tc.batch_ipv4_tx_fill(arena, d, pk.size, total, want_flags=False)
            tc.batch_ipv4_tx_fill(arena, d, pk.size, total, want_flags=False)  # idempotent
        np.testing.assert_array_equal(down(arena), want)


def test_pinned_host_arena_same_bytes(tc, torch, oracle):
    host, pk = _batch(tc, 7, 3)
    want = host.copy()
    oracle.batch_ipv4_tx_fill(want, pk, nthreads=8)
    arena = torch.from_numpy(host.copy()).pin_memory()  # written in place over PCIe
    d = tc.descs_to_device(pk)
    with tc.debug(tx_split=1):
        tc.batch_ipv4_tx_fill(arena, d, pk.size, int(pk["len"].sum()), want_flags=False)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(arena.numpy(), want)
