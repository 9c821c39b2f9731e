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

SOURCES = [os.path.join(CSRC, "csum_kernels.hip"), os.path.join(CSRC, "csum_api.cpp")]
HEADERS = [os.path.join(CSRC, "csum_launch.h")] + [
    os.path.join(INCLUDE, h) for h in ("tcsum.h", "tcsum_legacy.h", "tcsum_synth.h")]
# The capture-file helper (include/tcsum_pcap.h): host-only C++, a library of
# its own -- not part of the checksum path, so not in libtcsum.so.
PCAP_LIB = os.path.join(PKG, "libtcsum_pcap.so")
PCAP_SOURCES = [os.path.join(CSRC, "pcap_index.cpp")]
PCAP_HEADERS = [os.path.join(INCLUDE, h) for h in ("tcsum.h", "tcsum_pcap.h")]


def hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the gfx950 library cannot be built")


def _stale(lib: str, deps) -> bool:
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    return any(os.path.getmtime(p) > t for p in list(deps) + [__file__])


def stale() -> bool:
    return _stale(LIB, SOURCES + HEADERS) or _stale(PCAP_LIB, PCAP_SOURCES + PCAP_HEADERS)


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
    if _stale(PCAP_LIB, PCAP_SOURCES + PCAP_HEADERS) or not os.path.exists(PCAP_LIB):
        tmp = PCAP_LIB + ".tmp"
        cmd = [os.environ.get("CXX", "g++"), "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread", "-Wall",
               f"-I{INCLUDE}", PCAP_SOURCES[0], "-o", tmp]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        os.replace(tmp, PCAP_LIB)
    if not _stale(LIB, SOURCES + HEADERS):
        return LIB
    tmp = LIB + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-Wno-unused-function", f"-I{INCLUDE}", f"-I{CSRC}",
           "-x", "hip", SOURCES[0], "-x", "hip", SOURCES[1], "-o", tmp]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
