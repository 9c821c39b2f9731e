#!/bin/bash
# round 4, after the live-stack fixes: the GPU suite (integration tests
# included) and configs[0] timed again
set -u
out=gpurun_out/r04/final2
mkdir -p $out
scripts/gpu_steps.sh \
  "suite:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest_gpu.log 2>&1" \
  "configs0:400:scripts/configs0_timing.sh $out"
