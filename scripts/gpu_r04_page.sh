#!/bin/bash
# round 4: tcsum_host_batch_peso's pageable staging -- GPU suite (both forms
# of the pageable copy), smoke, and the pageable / pinned A/B
set -u
out=gpurun_out/r04/page
mkdir -p $out
scripts/gpu_steps.sh \
  "suite:700:python -u -m pytest tests -m gpu --maxfail=5 -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider > $out/pytest_gpu.log 2>&1" \
  "smoke:200:python -u -c 'import __graft_entry__ as g; g.smoke()' > $out/smoke.log 2>&1" \
  "ab:300:python -u scripts/e2e_pageable_probe.py > $out/e2e_pageable.txt 2>&1"
