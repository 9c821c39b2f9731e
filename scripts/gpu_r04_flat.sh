#!/bin/bash
# round 4: byte-window stream parity + one-process A/B against k_ipv4
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_flat.py -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/pytest_flat.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_flat.log
# 0 passed, 1 failed assertions: go on to the timings; anything else (a crash, a time limit): stop
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for cfg in mixed mixed_aligned mixed_rx mixed_txo mixed_tx; do
    timeout -k 10 240 python -u scripts/env_ab.py $cfg flat=1 >> gpurun_out/flat_ab.txt 2>&1 || exit $?
done
cat gpurun_out/flat_ab.txt
exit $rc
