#!/bin/bash
# usage: gpurun_wait.sh <logfile> <timeout> <cmd...>   -- retries only while gpurun reports exit 3 (no slot / box; nothing ran)
LOG=$1; shift; TO=$1; shift
for i in $(seq 1 40); do
    timeout $((TO + 900)) /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
    rc=$?
    echo "exit $rc (try $i)" >> "$LOG"
    [ $rc -ne 3 ] && exit $rc
    sleep 150
done
