#!/bin/bash
# PMC traffic (bench.py's own FETCH_SIZE / WRITE_SIZE passes) and kernel-trace
# fraction for every configuration, one bench line each.
set -u
out=${1:-gpurun_out/r02pmc}
mkdir -p "$out"
export TMPDIR=/tmp
cd "$(dirname "$0")/.." || exit 1
specs=()
for cfg in mtu tso mixed mixed_aligned mixed_tx mixed_txo mixed_rx; do
  specs+=("pmc_$cfg:300:TCSUM_PMC_KEEP=$out python -u bench.py --config $cfg --secondary '' --no-cpu --no-e2e > $out/bench_$cfg.json")
done
scripts/gpu_steps.sh "${specs[@]}"
