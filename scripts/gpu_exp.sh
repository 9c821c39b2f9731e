#!/bin/bash
# Round-2 experiments in one GPU call: the GPU suite, then header-load policy
# A/B (time, and HBM traffic through bench.py's own PMC passes), then the
# default bench line with the product-shaped probes.
set -u
out=${1:-gpurun_out/r02d}
mkdir -p "$out"
export TMPDIR=/tmp
cd "$(dirname "$0")/.." && scripts/gpu_steps.sh \
  "pytest:600:python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread" \
  "ab_rx:180:python -u scripts/env_ab.py mixed_rx TCSUM_IP_HDR_NT=1 > $out/ab_hdr_nt_rx.txt" \
  "ab_sums:180:python -u scripts/env_ab.py mixed TCSUM_IP_HDR_NT=1 > $out/ab_hdr_nt_sums.txt" \
  "ab_tx:180:python -u scripts/env_ab.py mixed_tx TCSUM_IP_HDR_NT=1 > $out/ab_hdr_nt_tx.txt" \
  "pmc_mixed:300:TCSUM_PMC_KEEP=$out/default python -u bench.py --config mixed --secondary '' --no-cpu --no-e2e --no-trace > $out/bench_mixed.json" \
  "pmc_mixed_nt:300:TCSUM_IP_HDR_NT=1 TCSUM_PMC_KEEP=$out/hdr_nt python -u bench.py --config mixed --secondary '' --no-cpu --no-e2e --no-trace > $out/bench_mixed_hdr_nt.json" \
  "bench:420:TCSUM_PMC_KEEP=$out python -u bench.py > $out/bench.json"
