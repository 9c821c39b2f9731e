#!/bin/bash
# Host-code sanitizers on the CPU tests (build container only; the kernels are
# not instrumented: -fsanitize= goes to the host side via -Xarch_host).
# Builds libtcsum.so with ASan + UBSan into a temp dir, swaps it in for the
# CPU suite's ABI / capture-file tests, and restores the normal build.
set -euo pipefail
cd "$(dirname "$0")/.."
tmp=$(mktemp -d)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -shared -Wno-unused-function \
    -Iinclude -Itcp_amd/csrc -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
    -Xarch_host -fno-omit-frame-pointer -shared-libsan \
    -x hip tcp_amd/csrc/csum_kernels.hip -x hip tcp_amd/csrc/csum_api.cpp \
    -Wl,--version-script=tcp_amd/csrc/libtcsum.map -o "$tmp/libtcsum.so"
cp tcp_amd/libtcsum.so "$tmp/libtcsum_normal.so"
trap 'cp "$tmp/libtcsum_normal.so" tcp_amd/libtcsum.so; touch tcp_amd/libtcsum.so; rm -rf "$tmp"' EXIT
cp "$tmp/libtcsum.so" tcp_amd/libtcsum.so
rt=$(/opt/rocm/lib/llvm/bin/clang++ -print-file-name=libclang_rt.asan-x86_64.so)
ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 LD_PRELOAD="$rt" \
    python -m pytest tests/test_abi.py tests/test_pcap.py tests/test_host_plan.py -x -q -m "not gpu" -p no:cacheprovider
