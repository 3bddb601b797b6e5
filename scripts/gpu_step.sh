#!/bin/bash
# Run one GPU step under its own time limit; stop the whole GPU call on a fault/abort/timeout
# (rc >= 124: timeout 124/137, abort 134, segfault 139) but continue after ordinary failures.
# usage: scripts/gpu_step.sh SECONDS LOGFILE cmd...
secs=$1; log=$2; shift 2
timeout -k 10 "$secs" "$@" > "$log" 2>&1
rc=$?
echo "[gpu_step] rc=$rc: $*" >> "$log"
if [ $rc -ge 124 ]; then echo "FATAL rc=$rc in: $*"; exit $rc; fi
exit 0
