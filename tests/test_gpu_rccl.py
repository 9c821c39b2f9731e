"""The bench's collectives over RCCL (torch.distributed backend "nccl" on
ROCm): a one-rank process group bound to the box's GPU, as tcp_amd.dist.init
binds one at N > 1, runs the three helpers bench.py uses -- barrier,
max_over_ranks on a device tensor, gather_objects -- and a device
all_reduce.  The N > 1 paths themselves are covered over gloo
(test_bench_launcher.py); a one-GPU box cannot hold two RCCL ranks."""
import os
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent("""
    import sys
    sys.path.insert(0, %r)
    import torch
    import torch.distributed as td
    from tcp_amd import dist as D
    torch.cuda.set_device(0)
    td.init_process_group("nccl", device_id=torch.device("cuda", 0))
    assert td.get_backend() == "nccl"
    D.barrier(td)
    assert D.max_over_ranks(td, 2.5, device="cuda") == 2.5
    assert D.gather_objects(td, {"rank": 0, "ms": 1.25}) == [{"rank": 0, "ms": 1.25}]
    t = torch.arange(4, dtype=torch.float32, device="cuda")
    td.all_reduce(t)
    torch.cuda.synchronize()
    assert t.tolist() == [0.0, 1.0, 2.0, 3.0]
    td.destroy_process_group()
    print("rccl ok")
""") % ROOT


def test_one_rank_rccl_group_runs_the_bench_collectives():
    from tcp_amd import dist as D
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", LOCAL_WORLD_SIZE="1",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(D.free_port()))
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "rccl ok" in r.stdout
