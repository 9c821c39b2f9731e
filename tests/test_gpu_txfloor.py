"""The tx fill's floor probe (libtcsum_bench.so, tcsum_probe_txfloor; in
stream, deferred, and deferred after loading each field's dword): it must
write exactly the bytes the fill writes --
each packet's IPv4 header checksum field (ipv4.c:643,656) and its TCP / UDP /
ICMP field (tcp_out.c:19-20, udp.c:320-321, icmpv4.c:45-58) -- and nothing
else, or the floor it prices is not the fill's.  The field addresses come
from its prepare pass; the expected ones from the product's tx offload (the
fields tcsum_tx_apply writes).  Measurement code, so the check is on
addresses, not values (the probe writes junk)."""
from devcopy import down, up
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


def _batch(tc, seed):
    from test_gpu_flat import _arena, _headers, _pk, _stream
    rng = np.random.default_rng(seed)
    lens = rng.integers(20, 9000, 700).astype(np.int64)
    short = rng.random(lens.size) < 0.1
    lens[short] = rng.integers(0, 20, int(short.sum()))
    offs = _stream(lens, 5)
    host = _arena(rng, int(offs[-1] + lens[-1]) + 512)
    _headers(rng, host, offs, lens, valid=0.9)
    return host, _pk(tc, offs, lens)


def _written(tc, torch, host, pk):
    """Byte positions the fill writes: apply all-zero and all-one values
    through the product's offload flags and see which bytes differ."""
    arena = up(torch.from_numpy(host.copy()))
    d = tc.descs_to_device(pk)
    _, fl = tc.batch_ipv4_tx_offload(arena, d, pk.size, int(pk["len"].sum()))
    fl = down(fl)
    a, b = host.copy(), host.copy()
    tc.tx_apply_batch(a, pk, np.zeros(pk.size, np.uint32), fl)
    tc.tx_apply_batch(b, pk, np.full(pk.size, 0xFFFFFFFF, np.uint32), fl)
    return set(np.nonzero(a != b)[0].tolist())


@pytest.mark.parametrize("seed", range(4))
def test_txfloor_writes_the_fills_fields(tc, torch, seed):
    host, pk = _batch(tc, seed)
    expect = _written(tc, torch, host, pk)
    assert expect, "the batch has fields to fill"
    for variant in (0, 1, 11):
        arena = torch.zeros(host.size + 256, dtype=torch.uint8, device="cuda")
        arena[: host.size] = up(torch.from_numpy(host))
        d = tc.descs_to_device(pk)
        h = tc.txfloor_prepare(arena, host.size, d, pk.size, int(pk["len"].sum()))
        fpos = down(h["fpos"])
        field = set()
        for f in fpos[fpos >= 0].tolist():
            field |= {f, f + 1}
        assert field == expect
        # each window's first packet: packets starting in it, in arena order
        ff = down(h["ffirst"])
        w = pk["offset"] // 16384
        for k in range(ff.size - 1):
            assert ff[k] == np.searchsorted(w, k, side="left")
        for _ in range(3):  # any number of launches touches only the fields
            tc.probe_txfloor(h, variant=variant)
        torch.cuda.synchronize()
        after = down(arena)
        changed = set(np.nonzero(after[: host.size] != host)[0].tolist())
        assert changed <= expect
        assert not after[host.size:].any()


def test_txfloor_refuses_short_buffers(tc, torch):
    from tcp_amd import _lib
    L = _lib.bench_lib()
    arena = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
    pk = np.zeros(4, tc.PKT_DTYPE)
    d = tc.descs_to_device(pk)
    side = torch.zeros(8, dtype=torch.uint32, device="cuda")
    fpos = torch.zeros(8, dtype=torch.int64, device="cuda")
    nw = L.tcsum_probe_txfloor_windows(1 << 16)
    assert nw == 4
    ff = torch.zeros(nw + 1, dtype=torch.uint32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    args = [arena.data_ptr(), 1 << 16, d.data_ptr(), 4, 0]
    assert L.tcsum_probe_txfloor_prepare(*args, side.data_ptr(), 7, fpos.data_ptr(), 8, ff.data_ptr(), nw + 1, s) != 0
    assert L.tcsum_probe_txfloor_prepare(*args, side.data_ptr(), 8, fpos.data_ptr(), 7, ff.data_ptr(), nw + 1, s) != 0
    assert L.tcsum_probe_txfloor_prepare(*args, side.data_ptr(), 8, fpos.data_ptr(), 8, ff.data_ptr(), nw, s) != 0
    assert L.tcsum_probe_txfloor_prepare(*args, side.data_ptr(), 8, fpos.data_ptr(), 8, ff.data_ptr(), nw + 1, s) == 0
    torch.cuda.synchronize()
