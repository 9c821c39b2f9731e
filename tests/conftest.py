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
