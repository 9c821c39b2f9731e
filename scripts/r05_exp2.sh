#!/bin/bash
# round 5: the packed kernel's scalar descriptors (parity, A/B, PMC), the
# fallback prefetch default, and the mixed line's order experiment
set -u
out=gpurun_out/r05d
mkdir -p $out
scripts/gpu_steps.sh \
  "variants:300:python -u -m pytest tests/test_gpu_prefetch.py -q --timeout 120 --timeout-method thread" \
  "pk_layouts:420:python -u scripts/pk_layouts_ab.py mtu,shuffled,ragged,small,big packed=0 lib=abl/libtcsum_r04.so pk_sdesc=1 pf_dist=0 > $out/pk_layouts_sdesc.txt" \
  "bench_def:400:TCSUM_PMC_KEEP=$out/pmc_def python -u bench.py --secondary '' --no-cpu --no-e2e > $out/bench_mtu_default.json" \
  "bench_sdesc:400:TCSUM_PMC_KEEP=$out/pmc_sdesc python -u bench.py --secondary '' --no-cpu --no-e2e --knob pk_sdesc=1 > $out/bench_mtu_sdesc.json" \
  "order:900:python -u scripts/bench_order_ab.py 2 > $out/bench_order_ab.txt"
