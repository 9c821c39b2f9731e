#!/bin/bash
# GPU call: suite, then A/B of three builds on the IPv4 modes.
set -u
out=${1:-gpurun_out/r02f}
mkdir -p "$out"
export TMPDIR=/tmp
cd "$(dirname "$0")/.." && scripts/gpu_steps.sh \
  "pytest:600:python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
  "ab:300:python -u scripts/ab_lib.py ab_libs/lib_a.so ab_libs/lib_c.so mixed,mixed_tx,mixed_rx > $out/ab_a_c.txt" \
  "ab2:300:python -u scripts/ab_lib.py ab_libs/lib_b.so ab_libs/lib_c.so mixed,mixed_tx,mixed_rx > $out/ab_b_c.txt"
