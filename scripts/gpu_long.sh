#!/bin/bash
# Run one gpurun call; retry ONLY when the pool reports a transient
# infrastructure failure before anything ran (status=transient, nothing
# charged), waiting as long as the pool's back-off asks.  A command that ran
# and failed is never retried.
# Usage: scripts/gpu_long.sh TIMEOUT_S 'command'
limit=$1; shift
for attempt in $(seq 1 40); do
    rm -f gpurun_out/steps.log  # results of earlier calls stay (copy what counts to profiles/)
    out=$(timeout $((limit + 900)) /usr/local/graft/bin/gpurun --timeout "$limit" -- "$@" 2>&1)
    rc=$?
    echo "$out" | grep -v "every call sends" | tail -4
    if echo "$out" | grep -q "status=transient\|backing off\|stopped responding while\|no box or slot"; then
        wait_s=$(echo "$out" | grep -o "retry in [0-9]*s" | tail -1 | grep -o "[0-9]*")
        wait_s=$(( ${wait_s:-80} + 10 ))
        [ $wait_s -lt 90 ] && wait_s=90
        echo "[gpu_long.sh] transient (attempt $attempt), retrying in $wait_s s"
        sleep $wait_s
        continue
    fi
    exit $rc
done
exit 3
