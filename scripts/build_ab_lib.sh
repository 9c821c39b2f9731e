#!/bin/bash
# Build libtcsum.so of a git revision into abl/libtcsum_<name>.so for a
# one-process A/B against the working tree (scripts/ab_lib.py).
#   scripts/build_ab_lib.sh REV NAME
set -e
rev=$1; name=$2
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
git -C "$root" archive "$rev" tcp_amd/csrc include | tar -x -C "$tmp"
mkdir -p "$root/abl"
map=""
[ -f "$tmp/tcp_amd/csrc/libtcsum.map" ] && map="-Wl,--version-script=$tmp/tcp_amd/csrc/libtcsum.map"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-function \
    -I"$tmp/include" -I"$tmp/tcp_amd/csrc" -x hip "$tmp/tcp_amd/csrc/csum_kernels.hip" \
    -x hip "$tmp/tcp_amd/csrc/csum_api.cpp" $map -o "$root/abl/libtcsum_$name.so"
rm -rf "$tmp"
echo "$root/abl/libtcsum_$name.so"
