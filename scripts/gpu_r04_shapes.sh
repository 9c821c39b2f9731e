#!/bin/bash
# r04: k_ipv4's launch forms (workgroup size, 8 waves per SIMD) on configs[3]
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04
timeout -k 10 400 python -u scripts/ipv4_shape_ab.py mixed mixed_aligned mixed_rx > gpurun_out/r04/ipv4_shape_ab.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r04/ipv4_shape_ab.txt
