#!/bin/bash
# round 3, call H: the headline geometry re-checked on the current kernel
# (G=32 x U=3, G=64 x U=2, G=16 x U=8 against G=16 x U=6), and why the TSO
# secondary of the default bench reads slower than TSO's own bench.
set -u
out=gpurun_out/r03
mkdir -p $out
scripts/gpu_steps.sh \
  "mtu_geom:300:python -u scripts/env_ab.py mtu TCSUM_G=32,TCSUM_U=3 TCSUM_G=64,TCSUM_U=2 TCSUM_G=16,TCSUM_U=8 TCSUM_G=8,TCSUM_U=16 > $out/ab_mtu_geom.txt" \
  "tso_sec_plain:300:python -u bench.py --no-pmc --no-trace --no-cpu --no-e2e --secondary tso > $out/bench_tso_secondary_plain.json" \
  "tso_sec_full:400:python -u bench.py --no-pmc --no-trace --secondary tso > $out/bench_tso_secondary_full.json"
