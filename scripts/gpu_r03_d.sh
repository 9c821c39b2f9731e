#!/bin/bash
# round 3, call D: TSO shapes around the 16-wave / wave-contiguous winner of
# call C (profiles/r03/ab_tso_shapes.txt), and the XCD grouping for it.
set -u
out=gpurun_out/r03
mkdir -p $out
V="TCSUM_WGX=16/64/4 TCSUM_WGX=16/64/2 TCSUM_WGX=16/64/3 TCSUM_WGX=8/64/4 TCSUM_WGX=8/64/2 TCSUM_WGX=4/64/4 TCSUM_WGX=16/32/4 TCSUM_WGX=16/128/4 TCSUM_WGX=16/256/4 TCSUM_WGX=16/16/4 TCSUM_WGX=16/64/4,TCSUM_XCD=1 TCSUM_WGX=16/64/4,TCSUM_XCD=8 TCSUM_WGX=16/64/4,TCSUM_XCD=16 TCSUM_WGX=16/64/4,TCSUM_XCD=256"
scripts/gpu_steps.sh \
  "tso_ab2:500:python -u scripts/env_ab.py tso $V > $out/ab_tso_shapes2.txt" \
  "tso_ab2b:500:python -u scripts/env_ab.py tso $V > $out/ab_tso_shapes2b.txt"
