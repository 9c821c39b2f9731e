#!/bin/bash
# round 4: k_segments_pk's range-by-range path at the per-range kernel's load
# depth, A/B against HEAD's build and the per-range kernel (packed=0)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_packed.py -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/pytest_packed.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_packed.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 500 python -u scripts/pk_layouts_ab.py mtu,shuffled,shufsmall,shufs200,shuftiny,shufbig,shufragged \
    lib=abl/libtcsum_r04base.so packed=0 > gpurun_out/pk_ab2.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/pk_ab2.txt
exit $rc
