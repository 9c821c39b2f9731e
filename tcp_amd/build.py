"""Build libtcsum.so in-tree with hipcc for gfx950.

The library is the product: the C ABI in include/*.h, implemented by
csrc/csum_api.cpp over the hand-written kernels in csrc/csum_kernels.hip.
It is built in place (tcp_amd/libtcsum.so) so it travels with the repo
snapshot to the GPU box.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(ROOT, "include")
LIB = os.path.join(PKG, "libtcsum.so")
ARCH = "gfx950"

SOURCES = [os.path.join(CSRC, "csum_kernels.hip"), os.path.join(CSRC, "csum_api.cpp"),
           os.path.join(CSRC, "pcap_index.cpp")]
HEADERS = [os.path.join(CSRC, "csum_launch.h")] + [
    os.path.join(INCLUDE, h) for h in ("tcsum.h", "tcsum_legacy.h", "tcsum_synth.h")]


def hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the gfx950 library cannot be built")


def stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(p) > t for p in SOURCES + HEADERS + [__file__])


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not stale():
        return LIB
    import fcntl
    with open(LIB + ".lock", "w") as lk:  # ranks of one node build once, not N times at once
        fcntl.flock(lk, fcntl.LOCK_EX)
        if not force and not stale():
            return LIB
        return _build_locked(verbose)


def _build_locked(verbose: bool) -> str:
    tmp = LIB + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-Wno-unused-function", f"-I{INCLUDE}", f"-I{CSRC}",
           "-x", "hip", SOURCES[0], "-x", "hip", SOURCES[1], "-x", "hip", SOURCES[2], "-o", tmp]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
