#!/bin/bash
# round 5: per-range kernel prefetch; the counters behind FETCH_SIZE
set -u
out=gpurun_out/r05h
mkdir -p $out
scripts/gpu_steps.sh \
  "variants:300:python -u -m pytest tests/test_gpu_prefetch.py -q --timeout 120 --timeout-method thread" \
  "pk_layouts:420:python -u scripts/pk_layouts_ab.py mtu,shuffled,shufsmall,ragged packed=0 packed=0,pf_range=1024 packed=0,pf_range=2048 pf_range=2048 > $out/pk_layouts_pfrange.txt" \
  "pmc_req:300:python -u scripts/pmc_requests.py $out > $out/pmc_requests.txt"
