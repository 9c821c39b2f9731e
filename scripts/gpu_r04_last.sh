#!/bin/bash
# round 4, the final tree: GPU suite and smoke
set -u
out=gpurun_out/r04/last
mkdir -p $out
scripts/gpu_steps.sh \
  "suite:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest_gpu.log 2>&1" \
  "smoke:200:python -u -c 'import __graft_entry__ as g; g.smoke()' > $out/smoke.log 2>&1"
