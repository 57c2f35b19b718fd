#!/bin/bash
# gpurun with a bounded retry when NO box could be had (exit 3 / "transient":
# nothing ran, nothing charged). A command that ran and failed is never retried.
# Usage: bash tools/gpurun_retry.sh <timeout-s> '<command>'
t=${1:?timeout}; shift
for a in 1 2 3 4 5 6; do
    out=$(/usr/local/graft/bin/gpurun --timeout "$t" -- "$@" 2>&1); rc=$?
    echo "$out" | tail -40
    if [ $rc -eq 3 ] || { echo "$out" | grep -q "status=transient"; }; then
        echo "# gpurun_retry: attempt $a had no box (rc $rc); waiting" >&2
        sleep 60
        continue
    fi
    exit $rc
done
exit 3
