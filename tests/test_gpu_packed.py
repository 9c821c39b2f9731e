"""k_segments_pk -- ranges packed back to back summed as one stream -- against
the oracle (the CPU restatement of net/src/tools.c:24-75 and
net/src/pktbuf.c:646-670, pinned to the reference's fixtures).

A workgroup streams the region from its first range's first byte to its
last range's end (pass by pass, up to 64 passes) when every one of its K
ranges lies inside that region; any other workgroup goes range by range.
Both paths and their mix inside one batch are checked bit for bit, with
ranges starting at every byte parity and chunk phase.
"""
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


@pytest.fixture(params=["packed"])
def packed(tc, request):
    """The stream kernel under test (debug knobs, include/tcsum_debug.h)."""
    tc.debug_set("packed", 1)
    yield request.param
    tc.debug_set("packed", -1)


def _arena(rng, size):
    host = rng.integers(0, 256, size, dtype=np.uint8)
    for _ in range(30):  # runs of 0x00 / 0xFF: sums of 0 and 0xFFFF
        a = int(rng.integers(0, size - 3000))
        host[a: a + int(rng.integers(1, 3000))] = rng.choice([0, 0xFF])
    return host


def _peso(tc, offs, lens, rng):
    p = np.zeros(len(lens), tc.PESO_DTYPE)
    p["offset"], p["len"] = offs, lens
    p["src"] = rng.integers(0, 256, (len(lens), 4))
    p["dst"] = rng.integers(0, 256, (len(lens), 4))
    p["protocol"] = rng.choice([6, 17], len(lens))
    return p


def _packed_offs(lens, start):
    return start + np.concatenate([[0], np.cumsum(lens[:-1])]).astype(np.uint64)


@pytest.mark.parametrize("start", [0, 1, 7, 12, 15])
@pytest.mark.parametrize("n", [1, 2, 42, 43, 44, 86, 4097])
def test_packed_mtu_vs_oracle(tc, torch, oracle, packed, n, start):
    """1500-B ranges packed from an arbitrary first byte (odd starts: every
    other range starts at an odd address); n around multiples of K = 43."""
    rng = np.random.default_rng(n * 16 + start)
    lens = np.full(n, 1500, np.uint32)
    host = _arena(rng, start + 1500 * n + 4096)
    p = _peso(tc, _packed_offs(lens, start), lens, rng)
    out = tc.batch_peso(up(torch.from_numpy(host)), tc.descs_to_device(p), n, int(lens.sum()))
    np.testing.assert_array_equal(down(out), oracle.batch_peso(host, p, nthreads=8))


@pytest.mark.parametrize("seed", range(6))
def test_packed_ragged_lengths(tc, torch, oracle, packed, seed):
    """Packed ranges of 17..3000 B (odd lengths: the parity flips range by
    range), the hint's mean setting K; some workgroups' regions exceed 64 KiB
    and take the per-range path."""
    rng = np.random.default_rng(500 + seed)
    n = 6000
    lens = rng.integers(17, 3001, n).astype(np.uint32)
    start = int(rng.integers(0, 64))
    host = _arena(rng, start + int(lens.sum()) + 4096)
    p = _peso(tc, _packed_offs(lens, start), lens, rng)
    hint = int(rng.choice([int(lens.sum()), 1500 * n, 700 * n]))  # K from the hint only
    out = tc.batch_peso(up(torch.from_numpy(host)), tc.descs_to_device(p), n, hint)
    np.testing.assert_array_equal(down(out), oracle.batch_peso(host, p, nthreads=8))


LAYOUTS = ["short", "tiny", "gap", "aligned", "overlap", "duplicate", "zero", "reversed", "far", "shuffled"]


@pytest.mark.parametrize("layout", LAYOUTS)
def test_packed_irregular_layouts(tc, torch, oracle, packed, layout):
    """Ranges that are not a clean packed stream.  Inside the region from the
    workgroup's first range to its last (short and 1..16-B ranges, gaps,
    16-B aligned starts, overlaps, duplicates, zero lengths) they are summed
    from the stream's prefixes; ranges outside it (descending order, a last
    range megabytes away, a shuffled batch) send the workgroup range by
    range."""
    rng = np.random.default_rng(LAYOUTS.index(layout))
    n = 43 * 40
    lens = np.full(n, 1500, np.int64)
    if layout == "tiny":
        lens = rng.integers(1, 17, n)
    offs = np.concatenate([[64], 64 + np.cumsum(lens[:-1])]).astype(np.int64)
    bad = rng.choice(n, 60, replace=False)
    if layout == "aligned":
        lens = rng.integers(1000, 2000, n)
        offs = 64 + np.concatenate([[0], np.cumsum((lens[:-1] + 15) // 16 * 16)])
    for i in bad:
        if layout == "short":
            lens[i] = int(rng.integers(1, 17))
        elif layout == "zero":
            lens[i] = 0
        elif layout == "gap":
            offs[i:] += int(rng.integers(1, 40))
        elif layout == "overlap":
            offs[i:] -= int(rng.integers(1, 40))
        elif layout == "duplicate" and i > 0:
            offs[i], lens[i] = offs[i - 1], lens[i - 1]
        elif layout == "far":
            offs[i] += 8 << 20
    if layout == "reversed":
        offs = offs[::-1].copy()
    if layout == "shuffled":
        perm = rng.permutation(n)
        offs, lens = offs[perm], lens[perm]
    host = _arena(rng, int((offs + lens).max()) + 4096)
    p = _peso(tc, offs.astype(np.uint64), lens.astype(np.uint32), rng)
    out = tc.batch_peso(up(torch.from_numpy(host)), tc.descs_to_device(p), n, int(lens.sum()))
    np.testing.assert_array_equal(down(out), oracle.batch_peso(host, p, nthreads=8))


@pytest.mark.parametrize("hint_mean", [300, 1500, 9000])
def test_packed_multi_pass_regions(tc, torch, oracle, packed, hint_mean):
    """Regions longer than one pass (ranges up to 70 KB; K from a small hinted
    mean), streamed pass by pass with the next pass's loads in flight; and
    regions over the pass limit, range by range."""
    rng = np.random.default_rng(hint_mean)
    n = 900
    lens = np.where(rng.random(n) < 0.2, rng.integers(20000, 70000, n), rng.integers(1, 3000, n)).astype(np.uint32)
    start = int(rng.integers(0, 16))
    host = _arena(rng, start + int(lens.sum()) + 4096)
    p = _peso(tc, _packed_offs(lens, start), lens, rng)
    out = tc.batch_peso(up(torch.from_numpy(host)), tc.descs_to_device(p), n, hint_mean * n)
    np.testing.assert_array_equal(down(out), oracle.batch_peso(host, p, nthreads=8))


def test_packed_long_range_word_sum_past_2_32(tc, torch, oracle, packed):
    """A 200-KB range of 0xFF bytes among 1500-B ones: its word sum exceeds
    2^32, where the stream's u32 prefix differences stop being exact -- its
    workgroup must sum range by range (ranges of 128 KiB and longer)."""
    rng = np.random.default_rng(17)
    n = 300
    lens = np.full(n, 1500, np.uint32)
    lens[[37, 150]] = [200000, 131071]
    host = _arena(rng, int(lens.sum()) + 4096)
    offs = _packed_offs(lens, 3)
    for i in (37, 150):
        host[int(offs[i]): int(offs[i]) + int(lens[i])] = 0xFF
    p = _peso(tc, offs, lens, rng)
    out = tc.batch_peso(up(torch.from_numpy(host)), tc.descs_to_device(p), n, 1500 * n)
    np.testing.assert_array_equal(down(out), oracle.batch_peso(host, p, nthreads=8))


@pytest.mark.parametrize("comp", [0, 1])
def test_packed_segments_mode(tc, torch, oracle, packed, comp):
    """tcsum_batch_segments (pktbuf_checksum16: u16 pre_sum, optional
    complement) on packed ranges."""
    rng = np.random.default_rng(31 + comp)
    n = 5000
    lens = rng.integers(900, 2200, n).astype(np.uint32)
    host = _arena(rng, 3 + int(lens.sum()) + 4096)
    s = np.zeros(n, tc.SEG_DTYPE)
    s["offset"], s["len"] = _packed_offs(lens, 3), lens
    s["pre_sum"] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    out = tc.batch_segments(up(torch.from_numpy(host)), tc.descs_to_device(s), n, comp, int(lens.sum()))
    np.testing.assert_array_equal(down(out), oracle.batch_segments(host, s, comp, nthreads=8))


def test_packed_exact_region_edges(tc, torch, oracle, packed):
    """Regions that end exactly on a chunk boundary (the end prefix is the
    last chunk's whole sum) and that fill the 64-KiB pass to the byte."""
    rng = np.random.default_rng(3)
    # K = 63 for mean 1040; 63 x 1040 = 65,520 B: with start 0 the region ends
    # chunk-aligned; 16 + 65,520 = the whole pass
    for start, L in ((0, 1040), (16, 1040), (1, 1040), (0, 1024), (8, 1488)):
        n = 63 * 5 + 1
        lens = np.full(n, L, np.uint32)
        host = _arena(rng, start + L * n + 4096)
        p = _peso(tc, _packed_offs(lens, start), lens, rng)
        out = tc.batch_peso(up(torch.from_numpy(host)), tc.descs_to_device(p), n, L * n)
        np.testing.assert_array_equal(down(out), oracle.batch_peso(host, p, nthreads=8))


def test_packed_full_mtu_config(tc, torch, oracle, packed):
    """configs[1] at full size (1M x 1500 B) through the packed kernel: every
    result equal to the oracle and to the per-range kernel."""
    from tcp_amd import workload
    b = workload.make_batch("mtu")
    arena, descs = workload.materialize(b)
    out = down(tc.batch_peso(arena, descs, b.n, b.total_bytes))
    np.testing.assert_array_equal(out, oracle.batch_peso(down(arena), b.descs, nthreads=16))


@pytest.mark.parametrize("seed", range(16))
def test_packed_fuzz(tc, torch, oracle, seed):
    """Seeded fuzz over the default shape: batches built from runs of packed
    ranges, gaps, overlaps, zero and 1..16-B ranges, long ranges (up to
    200 KB), descending and shuffled stretches, at random arena phases, with
    random length hints (K) -- checksum_peso and pktbuf_checksum16 (random
    pre_sum and complement) against the oracle."""
    rng = np.random.default_rng(4242 + seed)
    n = int(rng.integers(200, 4000))
    kind = rng.integers(0, 10, n)
    lens = np.where(kind < 6, rng.integers(17, 3000, n),
                    np.where(kind < 8, rng.integers(0, 17, n),
                             np.where(kind < 9, rng.integers(3000, 20000, n), rng.integers(20000, 200000, n))))
    step = lens + np.where(rng.random(n) < 0.2, rng.integers(-40, 64, n), 0)
    offs = int(rng.integers(0, 64)) + np.concatenate([[0], np.cumsum(np.maximum(step[:-1], 0))])
    for _ in range(int(rng.integers(0, 4))):  # a shuffled or reversed stretch
        a = int(rng.integers(0, n - 1))
        b = min(n, a + int(rng.integers(2, 200)))
        idx = np.arange(a, b)
        perm = idx[::-1] if rng.random() < 0.5 else rng.permutation(idx)
        offs[a:b], lens[a:b] = offs[perm], lens[perm]
    size = int((offs + lens).max()) + 4096
    host = _arena(rng, size)
    arena = up(torch.from_numpy(host))
    hint = int(rng.choice([int(lens.sum()), 300 * n, 1500 * n, 4000 * n]))
    p = _peso(tc, offs.astype(np.uint64), lens.astype(np.uint32), rng)
    out = tc.batch_peso(arena, tc.descs_to_device(p), n, hint)
    np.testing.assert_array_equal(down(out), oracle.batch_peso(host, p, nthreads=8))
    s = np.zeros(n, tc.SEG_DTYPE)
    s["offset"], s["len"] = offs, lens
    s["pre_sum"] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    comp = int(rng.integers(0, 2))
    out = tc.batch_segments(arena, tc.descs_to_device(s), n, comp, hint)
    np.testing.assert_array_equal(down(out), oracle.batch_segments(host, s, comp, nthreads=8))


HINT_LAYOUTS = ["mtu", "shuffled", "ragged_gaps", "shuffled576", "shuffled4000"]


@pytest.mark.parametrize("layout", HINT_LAYOUTS)
def test_layout_hints_give_the_same_results(tc, torch, oracle, layout):
    """tcsum_batch's layout hint changes only the kernel, never a result --
    also when the caller's ORDERED promise is false (a shuffled batch).
    SHUFFLED takes the packed kernel for ~1.5-KiB-and-up ranges (K <= 8) and
    the per-range kernel below (shuffled576)."""
    rng = np.random.default_rng(HINT_LAYOUTS.index(layout) + 100)
    n = 20000
    if layout.startswith("shuffled") and layout != "shuffled":
        lens = np.full(n, int(layout[len("shuffled"):]), np.int64)
    else:
        lens = np.full(n, 1500, np.int64) if layout != "ragged_gaps" else rng.integers(1, 3000, n)
    offs = _packed_offs(lens, 5).astype(np.int64)
    if layout == "ragged_gaps":
        offs += np.cumsum(rng.integers(0, 40, n))
    host = _arena(rng, int(offs.max() + lens.max()) + 4096)
    p = _peso(tc, offs.astype(np.uint64), lens.astype(np.uint32), rng)
    if layout.startswith("shuffled"):
        p = p[rng.permutation(n)]
    want = oracle.batch_peso(host, p, nthreads=8)
    arena = up(torch.from_numpy(host))
    d = tc.descs_to_device(p)
    s = np.zeros(n, tc.SEG_DTYPE)
    s["offset"], s["len"] = p["offset"], p["len"]
    s["pre_sum"] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    ds = tc.descs_to_device(s)
    want_s = oracle.batch_segments(host, s, 1, nthreads=8)
    for lay in (tc.LAYOUT_UNKNOWN, tc.LAYOUT_ORDERED, tc.LAYOUT_SHUFFLED):
        out, _, _ = tc.batch(tc.OP_PESO, arena, d, n, total_bytes=int(lens.sum()), layout=lay)
        np.testing.assert_array_equal(down(out), want)
        out, _, _ = tc.batch(tc.OP_SEGMENTS_COMP, arena, ds, n, total_bytes=int(lens.sum()), layout=lay)
        np.testing.assert_array_equal(down(out), want_s)


SMALL_CASES = [(64, "shuffled"), (200, "shuffled"), (576, "shuffled"), (700, "shuffled"), (400, "shuffled"),
               (200, "half"), (576, "half"), (64, "packed"), (576, "packed"), (300, "zeros"), (160, "shuffled"),
               (250, "half"), (80, "shuffled")]


@pytest.mark.parametrize("mean,layout", SMALL_CASES)
@pytest.mark.parametrize("mode", ["peso", "segments"])
def test_small_ranges_unknown_layout(tc, torch, oracle, mean, layout, mode):
    """Ranges under ~750 B (K > 16 ranges per packed workgroup) with no
    layout hint, the router's own choice: fully shuffled (every workgroup
    range by range), half the workgroups shuffled (both paths in one launch),
    fully packed, and ranges of length 0; n never a multiple of K.  Every
    path equals the oracle; so does the per-range kernel the SHUFFLED hint
    takes for these lengths (4 x 1 .. 8 x 3 by the mean, launch_segments)."""
    r = tc.route(mean)
    assert r["packed"] > 16, r
    K = r["packed"]
    rng = np.random.default_rng(mean * 7 + SMALL_CASES.index((mean, layout)) * 131 + (mode == "peso"))
    n = K * 97 + int(rng.integers(1, K))
    lens = rng.integers(max(1, mean // 2), mean * 3 // 2 + 1, n).astype(np.uint32)
    if layout == "zeros":
        lens[rng.choice(n, n // 5, replace=False)] = 0
    start = int(rng.integers(0, 64))
    offs = _packed_offs(lens, start)
    if layout == "shuffled":
        perm = rng.permutation(n)
    elif layout == "half":  # every other workgroup's K ranges permuted among themselves
        perm = np.arange(n)
        for w in range(0, n // K, 2):
            perm[w * K:(w + 1) * K] = rng.permutation(perm[w * K:(w + 1) * K])
    else:
        perm = np.arange(n)
    host = _arena(rng, start + int(lens.sum()) + 4096)
    total = int(lens.sum())
    if mode == "peso":
        d = _peso(tc, offs, lens, rng)[perm]
        run = lambda: tc.batch_peso(up(torch.from_numpy(host)), tc.descs_to_device(d), n, total)  # noqa: E731
        want = oracle.batch_peso(host, d, nthreads=8)
    else:
        d = np.zeros(n, tc.SEG_DTYPE)
        d["offset"], d["len"] = offs, lens
        d["pre_sum"] = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
        d = d[perm]
        run = lambda: tc.batch_segments(up(torch.from_numpy(host)), tc.descs_to_device(d), n, 1, total)  # noqa: E731
        want = oracle.batch_segments(host, d, 1, nthreads=8)
    np.testing.assert_array_equal(down(run()), want)
    with tc.debug(packed=0):
        np.testing.assert_array_equal(down(run()), want)
