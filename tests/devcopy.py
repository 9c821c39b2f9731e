"""How the GPU tests move bytes between host and device.

Default: through pinned host memory -- up(): pin_memory() then .cuda();
down(): tcp_amd.to_host (a pinned tensor, or a 64-MiB pinned bounce buffer).
TCSUM_TEST_PAGEABLE=1 (the diagnostic suite of DESIGN.md §4): the runtime's
pageable copies in both directions and the library's pageable staging off
(debug knob page_stage = 0, conftest.py) -- round 4's configuration, the one
the five hipErrorIllegalAddress stops came in.
"""
import os

PAGEABLE = os.environ.get("TCSUM_TEST_PAGEABLE") == "1"


def up(t):
    """A host tensor on the GPU (synchronous, like .cuda())."""
    return t.cuda() if PAGEABLE else t.pin_memory().cuda()


def down(t):
    """A device tensor's values as a numpy array (synchronous, like
    .cpu().numpy()); a host tensor's as they are."""
    if PAGEABLE or t.device.type != "cuda":
        return t.cpu().numpy()
    from tcp_amd.csum import to_host
    return to_host(t)
