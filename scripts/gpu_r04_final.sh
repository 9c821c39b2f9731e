#!/bin/bash
# round 4, last tree of the round -- configs[0] timed (coalescing on / off /
# queue server, the pcap driver's batches), the GPU suite, smoke, the default
# bench line (PMC / trace children, CPU baseline, e2e, every secondary
# config) and rocprofv3 --kernel-trace --stats of the same bench.
set -u
out=gpurun_out/r04/final
mkdir -p $out
scripts/gpu_steps.sh \
  "configs0:400:scripts/configs0_timing.sh $out" \
  "suite:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest_gpu.log 2>&1" \
  "smoke:200:python -u -c 'import __graft_entry__ as g; g.smoke()' > $out/smoke.log 2>&1" \
  "profile:700:scripts/profile_round.sh $out" \
  "window:300:python -u scripts/window_probe.py > $out/window_probe.txt 2>&1"
