#!/bin/bash
# r04: the whole GPU suite, then configs[0] timed with tx coalescing on / off /
# queue server (scripts/configs0_timing.sh), then k_ipv4's launch forms
set -u
out=gpurun_out/r04/suite_c0
mkdir -p $out
scripts/gpu_steps.sh \
  "suite:700:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest_gpu.log 2>&1" \
  "configs0:500:scripts/configs0_timing.sh $out" \
  "shapes:400:python -u scripts/ipv4_shape_ab.py mixed mixed_aligned mixed_rx > $out/ipv4_shape_ab.txt 2>&1"
