import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    _pinned_cpu_copies()


def _pinned_cpu_copies():
    """Every CUDA tensor's `.cpu()` in these tests copies through pinned
    memory (tcp_amd.to_host_tensor), as every upload already goes through
    pin_memory(): the runtime's pageable copies, in both directions, are
    where the round-5 GPU suites stopped.  Same values, same
    shape and dtype, synchronous like `.cpu()`."""
    import torch

    from tcp_amd.csum import to_host_tensor
    plain = torch.Tensor.cpu
    if getattr(plain, "_pinned", False):
        return

    def cpu(self, *args, **kwargs):
        if self.device.type == "cuda" and not args and not kwargs:
            return to_host_tensor(self)
        return plain(self, *args, **kwargs)
    cpu._pinned = True
    torch.Tensor.cpu = cpu


@pytest.fixture(scope="session")
def oracle():
    from oracle import pyoracle

    pyoracle.build()
    return pyoracle


@pytest.fixture
def dbg():
    """Set libtcsum debug knobs (include/tcsum_debug.h) for one test:
    dbg(server_idle_ms=50, ...); every knob it touched is unset after."""
    import tcp_amd
    touched = []

    def set_(**kv):
        for k, v in kv.items():
            tcp_amd.debug_set(k, int(v))
            touched.append(k)
    yield set_
    for k in touched:
        tcp_amd.debug_set(k, -1)
