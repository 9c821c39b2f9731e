#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/flat_probe.py mixed > gpurun_out/flat_probe.txt 2>&1
rc=$?
grep -v amdgpu.ids gpurun_out/flat_probe.txt
exit $rc
