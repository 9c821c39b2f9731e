#!/bin/bash
# round 4: the GPU suite on the current tree (one process), log under gpurun_out/
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
exit $rc
