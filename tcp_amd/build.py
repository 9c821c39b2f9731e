"""Build the libraries in-tree with hipcc for gfx950.

libtcsum.so is the product: the C ABI of include/tcsum.h, tcsum_legacy.h and
tcsum_debug.h, implemented by csrc/csum_api.cpp over the hand-written kernels
of csrc/csum_kernels.hip (device code in csrc/csum_device.h).  Measurement
and test-data kernels (include/tcsum_synth.h) are libtcsum_bench.so
(csrc/bench_kernels.hip), the capture-file helper (include/tcsum_pcap.h)
libtcsum_pcap.so.  Built in place so they travel with the repo snapshot to
the GPU box.
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
HEADERS = [os.path.join(CSRC, h) for h in ("csum_launch.h", "csum_device.h", "libtcsum.map")] + [
    os.path.join(INCLUDE, h) for h in ("tcsum.h", "tcsum_legacy.h", "tcsum_debug.h")]
# measurement kernels and synthetic data: a library of their own, linked
# against libtcsum.so (its probes follow the product's route)
BENCH_LIB = os.path.join(PKG, "libtcsum_bench.so")
BENCH_SOURCES = [os.path.join(CSRC, "bench_kernels.hip")]
BENCH_HEADERS = [os.path.join(CSRC, h) for h in ("csum_launch.h", "csum_device.h", "libtcsum_bench.map")] + [
    os.path.join(INCLUDE, h) for h in ("tcsum.h", "tcsum_debug.h", "tcsum_synth.h")]
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
    return (_stale(LIB, SOURCES + HEADERS) or _stale(BENCH_LIB, BENCH_SOURCES + BENCH_HEADERS + [LIB])
            or _stale(PCAP_LIB, PCAP_SOURCES + PCAP_HEADERS))


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not stale():
        return LIB
    import fcntl
    with open(LIB + ".lock", "w") as lk:  # ranks of one node build once, not N times at once
        fcntl.flock(lk, fcntl.LOCK_EX)
        if not force and not stale():
            return LIB
        return _build_locked(verbose, force)


def _hip_cmd(sources, out, mapfile, extra=()):
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wall", "-Wno-unused-function", f"-I{INCLUDE}", f"-I{CSRC}"]
    for src in sources:
        cmd += ["-x", "hip", src]
    return cmd + [f"-Wl,--version-script={mapfile}", *extra, "-o", out]


def _build_locked(verbose: bool, force: bool = False) -> str:
    if force or _stale(PCAP_LIB, PCAP_SOURCES + PCAP_HEADERS):
        tmp = PCAP_LIB + ".tmp"
        cmd = [os.environ.get("CXX", "g++"), "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread", "-Wall",
               f"-I{INCLUDE}", PCAP_SOURCES[0], "-o", tmp]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        os.replace(tmp, PCAP_LIB)
    if force or _stale(LIB, SOURCES + HEADERS):
        tmp = LIB + ".tmp"
        cmd = _hip_cmd(SOURCES, tmp, os.path.join(CSRC, "libtcsum.map"), ["-Wl,-soname,libtcsum.so"])
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        os.replace(tmp, LIB)
    if force or _stale(BENCH_LIB, BENCH_SOURCES + BENCH_HEADERS + [LIB]):
        tmp = BENCH_LIB + ".tmp"
        cmd = _hip_cmd(BENCH_SOURCES, tmp, os.path.join(CSRC, "libtcsum_bench.map"),
                       [f"-L{PKG}", "-l:libtcsum.so", "-Wl,-rpath,$ORIGIN"])
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        os.replace(tmp, BENCH_LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
