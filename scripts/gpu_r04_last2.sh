#!/bin/bash
# round 4, the final tree after the host_batch_peso diagnostics: GPU suite
# (up to 5 failures, each with its step and HIP error) and smoke
set -u
out=gpurun_out/r04/last2
mkdir -p $out
scripts/gpu_steps.sh \
  "suite:700:python -u -m pytest tests -m gpu --maxfail=5 -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest_gpu.log 2>&1" \
  "smoke:200:python -u -c 'import __graft_entry__ as g; g.smoke()' > $out/smoke.log 2>&1"
