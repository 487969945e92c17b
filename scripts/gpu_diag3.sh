#!/bin/bash
# Race screen with the GPU idled between launches (DIAG_SLEEP seconds): the rare differing launches
# were seen right after process start, i.e. on a GPU ramping up from idle.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TAG=${TAG:-s}
for i in $(seq 1 ${PROCS:-2}); do
  DIAG_SLEEP=${SLEEP:-0.2} DIAG_SAVE=gpurun_out/${TAG}_p$i.npz timeout -k 10 280 python -u scripts/diag_repeat.py ${N:-2} ${R:-200} > gpurun_out/${TAG}_p$i.log 2>&1 || { tail -5 gpurun_out/${TAG}_p$i.log; exit 1; }
  grep -E "runs differ|saved" gpurun_out/${TAG}_p$i.log
done
