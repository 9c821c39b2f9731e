#!/bin/bash
# One GPU call: the GPU test suite, then the judged bench lines with their
# PMC / kernel-trace children (raw CSVs kept), then the launcher checks.
# Usage (through gpurun): scripts/gpu_round.sh OUTDIR
set -u
out=${1:-gpurun_out/r02}
mkdir -p "$out"
export TMPDIR=/tmp
steps=(
  "pytest:600:python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread"
  "tx_probe:180:python -u scripts/tx_probe.py > $out/tx_probe.txt"
  "bench:420:TCSUM_PMC_KEEP=$out python -u bench.py > $out/bench.json"
  "bench_mixed_tx:300:TCSUM_PMC_KEEP=$out python -u bench.py --config mixed_tx --secondary '' --no-cpu --no-e2e > $out/bench_mixed_tx.json"
  "bench_mixed:300:TCSUM_PMC_KEEP=$out python -u bench.py --config mixed --secondary '' --no-cpu --no-e2e > $out/bench_mixed.json"
  "launcher_refuses:120:python -u bench.py --gpus 2 --steps 2 --warmup 1 > $out/launcher_refuses.txt 2>&1; test \$? -eq 2"
  "launcher_gloo2:300:TCSUM_DIST_BACKEND=gloo python -u bench.py --gpus 2 --no-pmc --no-trace --steps 20 > $out/launcher_gloo2.json"
)
cd "$(dirname "$0")/.." && scripts/gpu_steps.sh "${steps[@]}"
