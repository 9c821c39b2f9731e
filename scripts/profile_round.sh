#!/bin/bash
# Refresh the judged measurement set on the GPU box (run through gpurun):
#   1. the default bench line, with its own FETCH_SIZE / WRITE_SIZE PMC passes
#      (raw counter CSVs kept);
#   2. rocprofv3 --kernel-trace --stats of the same bench (--no-pmc: counters
#      cannot be collected under a tracing profiler), plus the trace grouped by
#      launch shape.
#      (--no-trace: the bench would otherwise start its own rocprofv3 child
#      under this one; --no-cpu --no-e2e: host-side legs, no kernels of note)
# Usage: scripts/profile_round.sh OUTDIR     (e.g. gpurun_out/prof)
# Every GPU step has its own time limit; the script stops at the first failure.
set -euo pipefail
out=${1:-gpurun_out/prof}
mkdir -p "$out"
export TMPDIR=/tmp
echo "== bench ($(date +%T))"
TCSUM_PMC_KEEP="$out" timeout -k 10 300 python -u bench.py > "$out/bench.json"
echo "== rocprof ($(date +%T))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/rocprof" -o bench \
    -- python -u bench.py --no-pmc --no-trace --no-cpu --no-e2e > "$out/bench_under_rocprof.json"
trace=$(find "$out/rocprof" -name 'bench_kernel_trace.csv' -print -quit)
stats=$(find "$out/rocprof" -name 'bench_kernel_stats.csv' -print -quit)
cp "$trace" "$out/bench_kernel_trace.csv"
cp "$stats" "$out/bench_kernel_stats.csv"
python scripts/group_trace.py "$out/bench_kernel_trace.csv" \
    "rocprofv3 --kernel-trace of \`python bench.py --no-pmc\`, grouped by kernel and grid" \
    > "$out/bench_kernel_by_launch.txt"
echo "== done ($(date +%T))"
