"""Packed-stream kernel (k_segments_pk) against the per-range kernels on
checksum_peso batches of several layouts, one process, interleaved rounds,
median us per launch; every variant's results must equal the default's.

  python scripts/pk_layouts_ab.py [LAYOUT,LAYOUT...] KEY=VALUE[,KEY=VALUE...] ...
  (KEY: a debug knob of include/tcsum_debug.h, or lib=PATH for another build)

Layouts (all ~1.5 GB, device-resident):
  mtu        configs[1]: 1M x 1500 B packed back to back
  shuffled   the same ranges, descriptor order permuted (not a packed stream)
  gaps       1500-B ranges with 0..63-B gaps between them
  ragged     packed, lengths uniform in 64..2936 B (mean 1500)
  small / big / tiny / s200 / j9000 / k16 / m1000 / m400   packed, 576 / 4000 / 64 / 200 / 9000 /
             16384 / 1000 / 400 B each; s40 / s72 / s80 / s100 / s128 / s160 / s250 / s320 / s440 / s480 / s530 / s640 likewise
  mixedlen   packed, lengths uniform in 64..9000 B
  shufNAME   any of the above with the descriptor order permuted (shufsmall, shufragged, ...)
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tcp_amd as tc  # noqa: E402
from tcp_amd.csum import PESO_DTYPE  # noqa: E402

variants = [{}] + [dict(kv.split("=", 1) for kv in a.split(",")) for a in sys.argv[1:] if "=" in a]
ROUNDS = int(os.environ.get("AB_ROUNDS", "8"))
TOTAL = 1500 << 20
rng = np.random.default_rng(7)


FIXED = {"mtu": 1500, "shuffled": 1500, "gaps": 1500, "small": 576, "big": 4000, "tiny": 64, "s200": 200,
         "j9000": 9000, "k16": 16384, "m1000": 1000, "m400": 400, "s40": 40, "s72": 72, "s80": 80, "s100": 100,
         "s128": 128, "s160": 160, "s250": 250, "s320": 320, "s640": 640, "s480": 480, "s440": 440, "s530": 530}
RAGGED = {"ragged": (64, 2937), "mixedlen": (64, 9001)}
NAMES = sys.argv[1].split(",") if len(sys.argv) > 1 and "=" not in sys.argv[1] else \
    ["mtu", "shuffled", "gaps", "ragged", "small", "big", "tiny", "s200", "j9000", "k16", "mixedlen"]


def layout(name):
    if name.startswith("shuf") and name != "shuffled":
        d, span = layout(name[4:])
        return d[rng.permutation(d.size)], span
    if name in FIXED:
        L = FIXED[name]
        lens = np.full(TOTAL // L, L, np.uint32)
    else:
        lo, hi = RAGGED[name]
        lens = rng.integers(lo, hi, TOTAL // ((lo + hi) // 2)).astype(np.uint32)
        lens = lens[np.cumsum(lens.astype(np.uint64)) <= TOTAL]
    gaps = rng.integers(0, 64, lens.size) if name == "gaps" else np.zeros(lens.size, np.int64)
    step = lens.astype(np.uint64) + gaps.astype(np.uint64)
    offs = np.concatenate([[0], np.cumsum(step[:-1])]).astype(np.uint64)
    d = np.zeros(lens.size, PESO_DTYPE)
    d["offset"], d["len"] = offs, lens
    d["src"] = rng.integers(0, 256, (lens.size, 4))
    d["dst"] = rng.integers(0, 256, (lens.size, 4))
    d["protocol"] = 6
    if name == "shuffled":
        d = d[rng.permutation(d.size)]
    return d, int(offs[-1] + lens[-1])


arena = torch.empty(TOTAL + (64 << 20), dtype=torch.uint8, device="cuda")
tc.synth_fill(arena)


OLD = {"TCSUM_G": "lanes", "TCSUM_U": "loads", "TCSUM_XCD": "xcd", "TCSUM_PACKED": "packed"}
_libs = {}


def with_env(env, fn):
    """A variant: lib=PATH runs another build of libtcsum.so (built by
    scripts/build_ab_lib.sh); every other KEY=VALUE is a debug knob
    (include/tcsum_debug.h; rounds 1-3's TCSUM_* names map to them)."""
    from tcp_amd import _lib
    prev = _lib._lib
    path = env.get("lib")
    if path:
        if path not in _libs:
            import ctypes
            L = ctypes.CDLL(os.path.abspath(path))
            for name, (res, args) in _lib.SIGNATURES.items():
                f = getattr(L, name, None)
                if f is not None:
                    f.restype, f.argtypes = res, args
            _libs[path] = L
        _lib._lib = _libs[path]
    knobs = {OLD.get(k, k): int(v) for k, v in env.items() if k != "lib"}
    try:
        if knobs and hasattr(_lib._lib, "tcsum_debug_set"):
            with tc.debug(**knobs):
                return fn()
        return fn()
    finally:
        _lib._lib = prev


for name in NAMES:
    d, span = layout(name)
    assert span <= arena.numel()
    dd = tc.descs_to_device(d)
    n, nb = d.size, int(d["len"].sum())
    outs = [torch.empty(n, dtype=torch.uint16, device="cuda") for _ in variants]

    def run(i):
        return with_env(variants[i], lambda: tc.batch_peso(arena, dd, n, nb, out=outs[i]))

    for i in range(len(variants)):
        for _ in range(5):
            run(i)
    torch.cuda.synchronize()
    ts = [[] for _ in variants]
    for r in range(ROUNDS):
        for k in range(len(variants)):  # the variant timed first rotates (the first of a round can run ~1 % slow)
            i = (r + k) % len(variants)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                run(i)
            e1.record()
            torch.cuda.synchronize()
            ts[i].append(e0.elapsed_time(e1) / 10 * 1e3)
    for i in range(1, len(variants)):
        assert torch.equal(outs[i], outs[0]), (name, variants[i])
    base = float(np.median(ts[0]))
    print(f"# {name}: {n} ranges, {nb} B", flush=True)
    for i, v in enumerate(variants):
        m = float(np.median(ts[i]))
        tag = ",".join(f"{k}={x}" for k, x in v.items()) or "default"
        print(f"  {tag:44s} {m:8.1f} us  {m / base:6.3f}x", flush=True)
    del dd, outs
