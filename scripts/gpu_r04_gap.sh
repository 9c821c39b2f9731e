#!/bin/bash
# round 4: why the default line's secondary configs read below their own
# dedicated lines -- the same line (no PMC / trace / e2e children) with the
# default 30-ms settle and with 300 ms (clocks after the CPU-baseline legs)
set -u
out=gpurun_out/r04/gap
mkdir -p $out
export TMPDIR=/tmp
scripts/gpu_steps.sh \
  "s30:300:python -u bench.py --no-pmc --no-trace --no-e2e > $out/bench_settle30.json" \
  "s300:300:python -u bench.py --no-pmc --no-trace --no-e2e --settle-ms 300 > $out/bench_settle300.json" \
  "nocpu:300:python -u bench.py --no-pmc --no-trace --no-e2e --no-cpu > $out/bench_nocpu.json"
