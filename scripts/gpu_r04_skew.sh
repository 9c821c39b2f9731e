#!/bin/bash
# r04: k_ipv4 with its data pass skewed 16 / 64 B past the packet's line (the
# window probe's finding), and the IPv4 parity tests on the rebuilt product
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "ipv4" -x -q --timeout 200 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/r04/pytest_ipv4.log 2>&1
rc=$?
tail -2 gpurun_out/r04/pytest_ipv4.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u scripts/ipv4_shape_ab.py mixed mixed_aligned mixed_rx --skew > gpurun_out/r04/ipv4_skew_ab.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r04/ipv4_skew_ab.txt
exit $rc
