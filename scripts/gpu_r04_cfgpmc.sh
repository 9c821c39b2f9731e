#!/bin/bash
# round 4, the last tree: every secondary config as its own bench line, each
# with its own FETCH_SIZE / WRITE_SIZE passes (HBM traffic per launch beside
# the algorithmic bytes) and trace child
set -u
out=gpurun_out/r04/cfgpmc
mkdir -p $out
export TMPDIR=/tmp
steps=()
for c in tso mixed mixed_aligned mixed_rx mixed_txo mixed_tx; do
  steps+=("$c:300:TCSUM_PMC_KEEP=$out python -u bench.py --config $c --secondary=, --no-cpu --no-e2e > $out/bench_$c.json")
done
scripts/gpu_steps.sh "${steps[@]}"
