#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04
timeout -k 10 400 python -u -m pytest tests/test_gpu_flat.py tests/test_gpu_packed.py -x -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/r04/pytest_hints.log 2>&1
rc=$?
tail -3 gpurun_out/r04/pytest_hints.log
exit $rc
