#!/bin/bash
# round 3, call F: the GPU suite on the current tree, and the headline shape
# with 16-wave workgroups / other XCD runs (one-process A/B).
set -u
out=gpurun_out/r03
mkdir -p $out
scripts/gpu_steps.sh \
  "pytest:400:python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread" \
  "mtu_ab:300:python -u scripts/env_ab.py mtu TCSUM_WG1024=1 TCSUM_WG1024=1,TCSUM_XCD=16 TCSUM_XCD=16 TCSUM_XCD=256 TCSUM_WG1024=1,TCSUM_XCD=256 > $out/ab_mtu_wg1024.txt" \
  "mixed_ab:300:python -u scripts/env_ab.py mixed TCSUM_XCD=16 TCSUM_XCD=256 TCSUM_G=16 TCSUM_WG1024=1 > $out/ab_mixed_xcd.txt"
