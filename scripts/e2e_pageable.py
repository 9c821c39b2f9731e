"""tcsum_host_batch_peso from pageable memory: the library's two pinned slots
(page_stage default) against the runtime's own pageable copy (page_stage=0),
and the pinned arena beside them; 1M x 1500 B (configs[1]'s batch).  Results
must agree across the three (measurement; the parity tests hold the oracle)."""
import ctypes
import time

import numpy as np

import tcp_amd as tc
from tcp_amd import _lib, workload


def timed(f, reps=5):
    f()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        out = f()
        ts.append(time.perf_counter() - t)
    return min(ts), sorted(ts)[len(ts) // 2], out


def main():
    b = workload.make_batch("mtu", n=1 << 20)
    nbytes = b.alloc_bytes
    rng = np.random.default_rng(7)
    page = rng.integers(0, 256, nbytes, dtype=np.uint8)
    segs = np.zeros(b.n, tc.PESO_DTYPE)
    segs["offset"], segs["len"] = b.descs["offset"], b.descs["len"]
    segs["src"] = rng.integers(0, 256, (b.n, 4))
    segs["dst"] = rng.integers(0, 256, (b.n, 4))
    segs["protocol"] = 6
    gib = float(segs["len"].sum()) / 2**30
    L = _lib.lib()
    p = L.tcsum_host_alloc(nbytes)
    assert p
    pinned = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p))
    pinned[:] = page
    res = {}
    try:
        for name, arena, stage in (("pinned", pinned, -1), ("pageable_slots", page, -1), ("pageable_runtime", page, 0)):
            tc.debug_set("page_stage", stage)
            lo, med, out = timed(lambda: tc.host_batch_peso(arena, segs))
            res[name] = out
            print(f"{name:18s} best {lo * 1e3:8.2f} ms  median {med * 1e3:8.2f} ms  {gib / lo:6.2f} GiB/s (best)", flush=True)
    finally:
        tc.debug_set("page_stage", -1)
        L.tcsum_host_free(p)
    same = all(np.array_equal(res["pinned"], v) for v in res.values())
    print("results equal across the three:", same, flush=True)
    assert same


if __name__ == "__main__":
    main()
