#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/flat_probe.py mixed > gpurun_out/flat_probe.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/flat_probe.txt
bash scripts/gpu_r04_pk.sh
