#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u scripts/cpu_baseline_repeat.py 3 4 > gpurun_out/r04/cpu_baseline_repeat.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r04/cpu_baseline_repeat.txt | tail -5
