"""Host-queue batches on pageable memory vs the same memory pinned in place
with tcsum_host_register (measurement script)."""
import sys, time, numpy as np
sys.path.insert(0, ".")
import tcp_amd as tc
from tcp_amd import workload
tc.plat_init(0)
for n in (50, 65536):
    b = workload.make_batch("mixed_tx", n=n)
    arena, descs = workload.materialize(b)
    raw = arena.cpu().numpy()
    del arena, descs
    reg = np.zeros(raw.size + 8192, np.uint8); a0 = (-reg.ctypes.data) % 4096
    region = reg[a0: a0 + (raw.size + 4095)//4096*4096]; region[:raw.size] = raw
    page = region.copy()
    reps = 200 if n <= 1024 else 10
    for name, arr, pin in (("pageable", page, False), ("registered", region, True)):
        if pin: tc.host_register(arr)
        for op in ("rx", "tx"):
            f = (lambda: tc.host_batch_ipv4_rx_verify(arr, b.descs)) if op == "rx" else (lambda: tc.host_batch_ipv4_tx_fill(arr, b.descs))
            f()
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter(); f(); ts.append(time.perf_counter() - t0)
            dt = float(np.median(ts))
            print(f"n={n:6d} {name:10s} {op}: {dt*1e6:9.1f} us  {b.total_bytes / dt / 2**30:6.2f} GiB/s", flush=True)
        if pin: tc.host_unregister(arr)
