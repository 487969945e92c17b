#!/bin/bash
# Race screen over many short processes (the rare differing launches cluster near process start):
# PROCS processes of R launches each; differing gradients saved to gpurun_out/ for offline analysis.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TAG=${TAG:-e}
for i in $(seq 1 ${PROCS:-8}); do
  DIAG_SAVE=gpurun_out/${TAG}_p$i.npz timeout -k 10 120 python -u scripts/diag_repeat.py ${N:-2} ${R:-40} > gpurun_out/${TAG}_p$i.log 2>&1 || { tail -5 gpurun_out/${TAG}_p$i.log; exit 1; }
  grep -E "runs differ|saved|sha1" gpurun_out/${TAG}_p$i.log
done
