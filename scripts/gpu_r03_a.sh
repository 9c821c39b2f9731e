#!/bin/bash
# round 3, call A: TSO load-shape A/B, the tx fill against its write-inclusive
# probe (with the calibrated traffic), and a quick default bench (devices +
# self_check).
set -u
out=gpurun_out/r03
mkdir -p $out
V="TCSUM_WGX=4/0/16 TCSUM_WGX=8/0/8 TCSUM_WGX=16/0/4 TCSUM_WGX=4/0/8 TCSUM_WGX=4/0/4 TCSUM_WGX=4/16/16 TCSUM_WGX=8/16/8 TCSUM_WGX=16/16/4 TCSUM_WGX=16/16/6 TCSUM_WGX=4/16/6 TCSUM_WGX=4/16/8 TCSUM_WGX=8/64/8 TCSUM_WGX=16/64/4"
scripts/gpu_steps.sh \
  "bench_quick:240:python -u bench.py --no-pmc --no-trace --no-cpu --no-e2e --secondary '' > $out/bench_quick.json" \
  "tso_ab:500:python -u scripts/env_ab.py tso $V > $out/ab_tso_shapes.txt" \
  "bench_tx:300:python -u bench.py --config mixed_tx --secondary '' --no-cpu --no-e2e --no-trace > $out/bench_mixed_tx.json"
