import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


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


@pytest.fixture(autouse=True)
def _device_drained(request):
    """After every GPU test: the whole device synchronized and its status
    checked -- every stream, the library's own and its resident servers
    included -- so a device fault is charged to the test whose work
    faulted, not to a later test's first HIP call."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import torch
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.synchronize()


@pytest.fixture(scope="session", autouse=True)
def _pageable_mode():
    """TCSUM_TEST_PAGEABLE=1: tcsum_host_batch_peso copies a pageable arena
    with the runtime's own pageable hipMemcpyAsync (debug knob page_stage =
    0), as it did in round 4 (devcopy.py)."""
    from devcopy import PAGEABLE
    if not PAGEABLE:
        yield
        return
    import tcp_amd
    tcp_amd.debug_set("page_stage", 0)
    yield
    tcp_amd.debug_set("page_stage", -1)
