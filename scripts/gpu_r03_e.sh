#!/bin/bash
# round 3, call E: the GPU suite with the 16-wave TSO kernel as the default
# (and its new geometry among the tested ones), the TSO bench line with its
# PMC / trace children, and the MTU A/B of the wave-contiguous multi-range
# kernel k_segments_wv.
set -u
out=gpurun_out/r03
mkdir -p $out
W="TCSUM_WV=4/4/6 TCSUM_WV=16/4/6 TCSUM_WV=8/4/6 TCSUM_WV=4/2/3 TCSUM_WV=16/2/3 TCSUM_WV=4/1/2 TCSUM_WV=16/1/2 TCSUM_WV=4/8/12 TCSUM_WV=4/3/5"
scripts/gpu_steps.sh \
  "pytest:400:python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread" \
  "mtu_ab:400:python -u scripts/env_ab.py mtu $W > $out/ab_mtu_wv.txt" \
  "bench_tso:400:TCSUM_PMC_KEEP=$out/pmc_tso python -u bench.py --config tso --secondary '' --no-cpu --no-e2e > $out/bench_tso.json"
