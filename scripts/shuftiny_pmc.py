"""Shuffled 64-B checksum_peso ranges (pk_layouts_ab.py's shuftiny) through
the packed kernel's range-by-range path and through the per-range kernel
(debug packed = 0), a few launches each, for rocprofv3 --pmc passes:
the two kernels' bytes from HBM side by side.  Measurement script.

  rocprofv3 --pmc FETCH_SIZE --kernel-trace ... -- python scripts/shuftiny_pmc.py
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tcp_amd as tc  # noqa: E402
from tcp_amd.csum import PESO_DTYPE  # noqa: E402

L = int(os.environ.get("SHUF_LEN", "64"))
TOTAL = 1500 << 20
rng = np.random.default_rng(7)
n = TOTAL // L
d = np.zeros(n, PESO_DTYPE)
d["offset"] = np.arange(n, dtype=np.uint64) * np.uint64(L)
d["len"] = L
d["protocol"] = 6
d = d[rng.permutation(n)]
arena = torch.empty(TOTAL + (64 << 20), dtype=torch.uint8, device="cuda")
tc.synth_fill(arena)
dd = tc.descs_to_device(d)
out = torch.empty(n, dtype=torch.uint16, device="cuda")
for packed in (-1, 0):
    with tc.debug(packed=packed):
        for _ in range(5):
            tc.batch_peso(arena, dd, n, n * L, out=out)
torch.cuda.synchronize()
print("done", n, flush=True)
