#!/bin/bash
# Run one gpurun call; retry ONLY when the pool reports a transient
# infrastructure failure before anything ran (status=transient, nothing
# charged).  A command that ran and failed is never retried.
# Usage: scripts/gpu.sh TIMEOUT_S 'command'
limit=$1; shift
for attempt in $(seq 1 40); do
    rm -f gpurun_out/steps.log  # results of earlier calls stay (copy what counts to profiles/)
    out=$(timeout $((limit + 900)) /usr/local/graft/bin/gpurun --timeout "$limit" -- "$@" 2>&1)
    rc=$?
    echo "$out" | tail -4
    if echo "$out" | grep -q "status=transient\|backing off\|stopped responding while\|no box or slot"; then
        echo "[gpu.sh] transient (attempt $attempt), retrying in 90 s"
        sleep 90
        continue
    fi
    exit $rc
done
exit 3
