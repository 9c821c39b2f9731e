#!/bin/bash
# r04: configs[0] timed with tx coalescing on / off / queue server, and the
# pcap driver's phases and batch sizes
set -u
out=gpurun_out/r04/c0
mkdir -p $out
scripts/gpu_steps.sh "configs0:600:scripts/configs0_timing.sh $out"
