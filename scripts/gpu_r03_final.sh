#!/bin/bash
# round 3: the judged set on the current tree -- smoke, the default bench line
# (with its PMC / trace children, CPU baseline, e2e, every secondary config),
# and rocprofv3 --kernel-trace --stats of the same bench.
set -u
out=gpurun_out/r03/final
mkdir -p $out
scripts/gpu_steps.sh \
  "smoke:200:python -u -c 'import __graft_entry__ as g; g.smoke()' > $out/smoke.log 2>&1" \
  "profile:700:scripts/profile_round.sh $out"
