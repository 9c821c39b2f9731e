#!/bin/bash
# round 3, call B: the integration GPU tests (loop echo, the pcap driver over
# the test double), configs[0] timing, counter calibration, a quick bench line.
set -u
out=gpurun_out/r03
mkdir -p $out
scripts/gpu_steps.sh \
  "itest:280:python -u -m pytest tests/test_integration.py -m gpu -v --timeout 250 --timeout-method thread" \
  "configs0:300:scripts/configs0_timing.sh $out" \
  "calib:240:python -u scripts/pmc_calib.py $out/pmc_calib.json" \
  "bench_quick:240:python -u bench.py --no-pmc --no-trace --no-cpu --no-e2e --secondary '' > $out/bench_quick.json"
