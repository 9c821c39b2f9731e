#!/bin/bash
# r04: the window stream's load phase with its prologue varied (what
# separates it from the TSO kernel on configs[3]'s arena)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04
timeout -k 10 500 python -u scripts/window_probe.py > gpurun_out/r04/window_probe.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r04/window_probe.txt
