#!/bin/bash
# r04: tx floor tests + the mixed_tx line with its floor; the flat stream
# against the packet-agnostic ceiling on configs[3]; k_segments_pk's
# per-range path on shuffled layouts
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_txfloor.py tests/test_gpu_packed.py -x -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_combo2.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_combo2.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --config mixed --secondary mixed_tx --no-pmc --no-cpu --no-e2e --no-trace \
    --steps 20 > gpurun_out/bench_tx.json 2> gpurun_out/bench_tx.err || exit $?
python -c "
import json; d=json.loads(open('gpurun_out/bench_tx.json').read().strip().splitlines()[-1])
for k,v in d.get('configs',{}).items(): print(k, json.dumps(v.get('roofline',{}))[:1200])" || true
timeout -k 10 400 python -u scripts/flat_probe.py mixed 4x3,8x4,16x4 0,1,2 extra > gpurun_out/flat_probe2.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/flat_probe2.txt
timeout -k 10 500 python -u scripts/pk_layouts_ab.py mtu,shuffled,shufsmall,shufs200,shuftiny,shufbig,shufragged \
    lib=abl/libtcsum_r04base.so packed=0 > gpurun_out/pk_ab2.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/pk_ab2.txt
exit $rc
