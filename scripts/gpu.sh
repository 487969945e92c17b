#!/bin/bash
# gpurun wrapper for this container: re-submits ONLY when the pool reports a transient failure in
# which no part of the command ran (no box acquired / box lost while being prepared); a command
# that ran and failed is never re-submitted.  Usage: scripts/gpu.sh <timeout-s> '<command>'
T=$1; shift
for attempt in 1 2 3; do
  out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1)
  rc=$?
  echo "$out" | grep -v "every call sends"
  if echo "$out" | grep -q "status=transient" && ! echo "$out" | grep -q "run [1-9]"; then
    echo "[gpu.sh] transient pool failure (nothing ran), retrying in 60 s"; sleep 60; continue
  fi
  exit $rc
done
exit 3
