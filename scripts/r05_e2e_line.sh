set -o pipefail
mkdir -p gpurun_out/r05e/line
for i in 1 2; do
  for pol in prealloc free; do
    timeout -k 10 400 python -u bench.py --no-pmc --no-trace --arena-policy $pol > gpurun_out/r05e/line/bench_${pol}_$i.json 2> gpurun_out/r05e/line/bench_${pol}_$i.err || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/r05e/line/bench_${pol}_$i.json').read().strip().splitlines()[-1]); e=d['e2e']; print('$pol $i', d['roofline']['frac'], e['gib_s'], e['h2d_copy_gib_s'], e['host_queue_rx']['gib_s'])"
  done
done
