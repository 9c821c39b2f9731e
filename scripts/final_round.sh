#!/bin/bash
# The round's last measurement set on the GPU box (run through gpurun):
#   GPU suite, smoke, the default bench line with its PMC passes and the
#   rocprofv3 --kernel-trace --stats set (scripts/profile_round.sh), and
#   bench.py --gpus 8 over gloo with the 8 ranks sharing this box's GPU (the
#   N = 8 path's wall time and line fields; not a scaling measurement).
# Usage: scripts/final_round.sh OUTDIR
# Every GPU step has its own time limit; the script stops at the first failure.
set -euo pipefail
out=${1:-gpurun_out/final}
mkdir -p "$out"
export TMPDIR=/tmp
echo "== pytest ($(date +%T))"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > "$out/pytest_gpu.log" 2>&1
echo "== smoke ($(date +%T))"
timeout -k 10 300 python -u -c 'import __graft_entry__ as g; g.smoke()' > "$out/smoke.log" 2>&1
bash scripts/profile_round.sh "$out"
echo "== 8 ranks over gloo on one GPU ($(date +%T))"
TCSUM_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 8 --steps 20 --warmup 5 \
    > "$out/bench_8ranks_gloo_one_gpu.json" 2> "$out/bench_8ranks_gloo_one_gpu.err"
echo "== done ($(date +%T))"
