#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_flat.py -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/pytest_flat.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_flat.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/flat_probe.py mixed 4x3,8x3,8x4 > gpurun_out/flat_probe.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/flat_probe.txt
exit $rc
