#!/bin/bash
# round 4, the last tree: the default bench line and its rocprofv3 children
# (confirms profiles/r04/final/ on the tree the round ends with)
set -u
out=gpurun_out/r04/last3
mkdir -p $out
scripts/gpu_steps.sh "profile:700:scripts/profile_round.sh $out"
