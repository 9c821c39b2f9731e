"""tcp_amd.to_host / to_host_tensor: device tensors read back through pinned
memory only, and the tests' read-back helper over it
(tests/devcopy.py)."""
import numpy as np
import pytest
from devcopy import down


def test_host_tensor_passes_through():
    import torch

    import tcp_amd as tc
    t = torch.arange(10, dtype=torch.int16)
    assert tc.to_host_tensor(t) is t
    np.testing.assert_array_equal(tc.to_host(t), np.arange(10, dtype=np.int16))


@pytest.mark.gpu
@pytest.mark.parametrize("n,dtype", [(0, "uint8"), (1, "uint16"), (4099, "uint32"), (70 << 20, "uint8"),
                                     ((20 << 20) + 7, "int32"), (3000, "bool")])
def test_to_host_values(n, dtype):
    """Small results in one pinned tensor, larger than 64 MiB through the
    bounce buffer (70 MiB of u8, 80 MiB of i32 with a ragged last chunk)."""
    import torch

    import tcp_amd as tc
    dt = getattr(torch, dtype)
    if dtype == "bool":
        d = (torch.arange(n, device="cuda") % 3) == 0
        want = (np.arange(n) % 3) == 0
    else:
        d = torch.arange(n, dtype=torch.int64, device="cuda").to(dt) if n else torch.empty(0, dtype=dt, device="cuda")
        want = np.arange(n, dtype=np.int64).astype(np.dtype(dtype))
    h = tc.to_host_tensor(d)
    assert h.device.type == "cpu" and h.dtype == dt and tuple(h.shape) == (n,)
    np.testing.assert_array_equal(h.numpy(), want)
    np.testing.assert_array_equal(down(d), want)  # the tests' read-back helper


@pytest.mark.gpu
def test_to_host_views():
    """Non-contiguous and offset views read back in their own shape."""
    import torch

    import tcp_amd as tc
    base = torch.arange(6 * 1000, dtype=torch.int32, device="cuda").reshape(6, 1000)
    want = np.arange(6 * 1000, dtype=np.int32).reshape(6, 1000)
    np.testing.assert_array_equal(tc.to_host(base.t()), want.T)
    np.testing.assert_array_equal(tc.to_host(base[2:5, 17:900]), want[2:5, 17:900])
    np.testing.assert_array_equal(tc.to_host(base[3, 5]), want[3, 5])
