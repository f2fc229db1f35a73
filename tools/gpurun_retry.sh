#!/bin/bash
# tools/gpurun_retry.sh LOG TIMEOUT 'command'  -- one gpurun call, re-queued only while the pool
# has no box or slot for it (nothing ran, nothing charged); any other outcome ends it.
log=$1; to=$2; cmd=$3
for i in $(seq 1 12); do
    /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
    rc=$?
    if grep -q "no free box right now\|slot(s) on this pod are busy\|stopped responding while being prepared\|is backing off" "$log"; then
        echo "[retry $i] $(date +%T) no box; waiting" >> "$log.retries"
        sleep 150
        continue
    fi
    exit $rc
done
exit 3
