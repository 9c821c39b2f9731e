#!/bin/bash
# round 4, the tree the round ends with: the default bench line (after the
# PMC step-kernel fix) and mixed_rx alone with its corrected traffic
set -u
out=gpurun_out/r04/end
mkdir -p $out
export TMPDIR=/tmp
scripts/gpu_steps.sh \
  "bench:420:python -u bench.py > $out/bench.json" \
  "rx:300:python -u bench.py --config mixed_rx --secondary=, --no-cpu --no-e2e > $out/bench_mixed_rx.json"
