#!/bin/bash
# round 3, call C: TSO load-shape A/B (one process, interleaved, results
# checked against the default kernel), and the loop echo with the queue server.
set -u
out=gpurun_out/r03
mkdir -p $out
V="TCSUM_WGX=4/0/16 TCSUM_WGX=8/0/8 TCSUM_WGX=16/0/4 TCSUM_WGX=4/0/8 TCSUM_WGX=4/0/4 TCSUM_WGX=4/16/16 TCSUM_WGX=8/16/8 TCSUM_WGX=16/16/4 TCSUM_WGX=16/16/6 TCSUM_WGX=4/16/6 TCSUM_WGX=4/16/8 TCSUM_WGX=8/64/8 TCSUM_WGX=16/64/4"
scripts/gpu_steps.sh \
  "tso_ab:500:python -u scripts/env_ab.py tso $V > $out/ab_tso_shapes.txt" \
  "echo_qs:120:for r in 1 2 3; do NET_CSUM_QUEUE_SERVER=1 integration/_build/loop_echo --rounds 2000 --tcp-bytes 1048576 | grep -E '^timing|^engine'; done > $out/configs0_queue_server.txt"
