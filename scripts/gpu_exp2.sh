#!/bin/bash
# GPU call: suite, A/B of two builds (line-aligned k_ipv4 passes), traffic, default bench.
set -u
out=${1:-gpurun_out/r02e}
mkdir -p "$out"
export TMPDIR=/tmp
cd "$(dirname "$0")/.." && scripts/gpu_steps.sh \
  "pytest:600:python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
  "ab:300:python -u scripts/ab_lib.py ab_libs/lib_a.so ab_libs/lib_b.so mixed,mixed_tx,mixed_rx > $out/ab_line_aligned.txt" \
  "pmc_mixed:300:TCSUM_PMC_KEEP=$out python -u bench.py --config mixed --secondary '' --no-cpu --no-e2e > $out/bench_mixed.json" \
  "bench:420:TCSUM_PMC_KEEP=$out python -u bench.py > $out/bench.json"
