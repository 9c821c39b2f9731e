#!/bin/bash
# Run GPU steps on the gpurun box; stop at the first crash or time-out.
# Usage: scripts/gpu_steps.sh NAME:LIMIT_S:COMMAND ...   (COMMAND is one shell word list)
# rc 0 = ok, rc 1 = ordinary failure (pytest failures / Python exception):
# keep going; anything else (abort, segfault, time-out) ends the call.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
    name=${spec%%:*}; rest=${spec#*:}; limit=${rest%%:*}; cmd=${rest#*:}
    echo "== $name ($(date +%T)) $cmd" >> gpurun_out/steps.log
    timeout -k 10 "$limit" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "== $name rc=$rc ($(date +%T))" >> gpurun_out/steps.log
    tail -5 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "stopping after $name (rc=$rc)"
        exit $rc
    fi
done
exit 0
