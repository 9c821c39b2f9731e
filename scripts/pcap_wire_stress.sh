#!/bin/bash
mkdir -p gpurun_out/stress
f=0
for i in $(seq 1 10); do
  timeout -k 10 60 integration/_build/pcap_wire tests/golden > gpurun_out/stress/pw_$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then f=$((f+1)); echo "run $i rc=$rc"; grep ": FAIL" gpurun_out/stress/pw_$i.log | head -2; fi
  if [ $rc -ge 124 ]; then break; fi
done
echo "gpu pcap_wire fails=$f/10"
