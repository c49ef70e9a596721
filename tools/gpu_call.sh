#!/bin/bash
# Submit one gpurun call; resubmit (after a pause) only when gpurun reports a
# transient pool condition (no free slot / box lost while being prepared) --
# never after the command itself ran.  Usage: tools/gpu_call.sh LOG TIMEOUT 'CMD'
LOG=$1
TMO=$2
CMD=$3
for i in 1 2 3 4 5 6 7 8; do
    timeout $((TMO + 900)) /usr/local/graft/bin/gpurun --timeout "$TMO" -- "$CMD" > "$LOG" 2>&1
    if grep -q "status=transient" "$LOG"; then
        echo "[gpu_call] transient pool condition (attempt $i); retrying in 150 s" >> "$LOG.attempts"
        sleep 150
        continue
    fi
    break
done
tail -20 "$LOG"
