#!/bin/bash
# r04: pk per-range path A/B (shuffled layouts), tx floor, and kernel traces
# of the flat probe and the mixed_tx bench (plan / scatter kernels and the
# gaps between a call's launches)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/c3
export TMPDIR=/tmp
o=gpurun_out/c3
timeout -k 10 300 python -u -m pytest tests/test_gpu_txfloor.py tests/test_gpu_packed.py -x -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider > $o/pytest.log 2>&1
rc=$?
tail -3 $o/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 500 python -u scripts/pk_layouts_ab.py mtu,shuffled,shufsmall,shuftiny,shufragged,ragged \
    lib=abl/libtcsum_r04base.so packed=0 > $o/pk_ab3.txt 2>&1 || exit $?
grep -v amdgpu.ids $o/pk_ab3.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/rp_tx -o tx -- \
    python -u bench.py --config mixed --secondary mixed_tx --no-pmc --no-cpu --no-e2e --no-trace --steps 20 \
    > $o/bench_tx.json 2> $o/bench_tx.err || exit $?
python -c "
import json; d=json.loads(open('$o/bench_tx.json').read().strip().splitlines()[-1])
for k,v in d.get('configs',{}).items(): print(k, v['ms_per_step'], json.dumps(v.get('roofline',{}).get('probes')))" || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/rp_flat -o flat -- \
    python -u scripts/flat_probe.py mixed 4x3,16x4 0,1 > $o/flat_probe3.txt 2>&1 || exit $?
grep -v amdgpu.ids $o/flat_probe3.txt
for f in $(find $o -name '*_kernel_stats.csv'); do echo "== $f"; cut -d, -f1-8 $f | head -20; done
exit $rc
