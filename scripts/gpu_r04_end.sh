#!/bin/bash
# round 4, the tree the round ends with: the default bench line (after the
# PMC step-kernel fix and the 300-ms settle)
set -u
out=gpurun_out/r04/end2
mkdir -p $out
export TMPDIR=/tmp
scripts/gpu_steps.sh \
  "bench:420:python -u bench.py > $out/bench.json"
  
