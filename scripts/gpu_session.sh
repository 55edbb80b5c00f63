#!/bin/bash
# Runs a sequence of GPU steps on the gpurun box; each step under its own
# time limit. Stops at the first step that faults / aborts / times out
# (exit 124, 134, 137, 139 or >128); ordinary test failures (exit 1) do not
# stop the session. Usage: scripts/gpu_session.sh TAG "cmd1" "cmd2" ...
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for cmd in "$@"; do
    i=$((i+1))
    echo "=== step $i: $cmd" | tee -a "$OUT/session.log"
    bash -c "$cmd" > "$OUT/step$i.log" 2>&1
    rc=$?
    echo "=== step $i rc=$rc" | tee -a "$OUT/session.log"
    tail -3 "$OUT/step$i.log" | tee -a "$OUT/session.log"
    if [ $rc -ge 124 ]; then
        echo "=== stopping after fatal rc=$rc" | tee -a "$OUT/session.log"
        exit $rc
    fi
done
exit 0
