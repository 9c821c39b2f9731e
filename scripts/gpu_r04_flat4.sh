#!/bin/bash
# r04: flat kernel (packets on wave 0), tx floor probe tests, flat probes,
# and the mixed_tx line with its floor
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_flat.py tests/test_gpu_txfloor.py -x -q --timeout 300 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_flat.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_flat.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/flat_probe.py mixed 4x3,8x3,8x4 > gpurun_out/flat_probe.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/flat_probe.txt
timeout -k 10 300 python -u bench.py --config mixed --secondary mixed_tx --no-pmc --no-cpu --no-e2e --no-trace \
    --steps 20 > gpurun_out/bench_tx.json 2> gpurun_out/bench_tx.err || exit $?
python -c "
import json; d=json.loads(open('gpurun_out/bench_tx.json').read().strip().splitlines()[-1])
for k,v in d.get('configs',{}).items(): print(k, json.dumps(v.get('roofline',{}))[:900])
print('head', json.dumps(d['roofline'])[:600])"
exit $rc
