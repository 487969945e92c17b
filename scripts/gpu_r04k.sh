#!/bin/bash
# round-4: save the distinct gradients of the race screen (sqnu665j 8x8, 4 images) for offline analysis
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for k in 1 2 3 4 5 6; do
  HPE_SPLIT_ONLY=1 DIAG_SLEEP=0.01 DIAG_SAVE=gpurun_out/r04k_$k.npz timeout -k 10 120 python -u scripts/diag_repeat.py 4 30 sqnu665j 8 > gpurun_out/r04k_$k.log 2>&1 || { tail -5 gpurun_out/r04k_$k.log; exit 1; }
  grep -E "runs differ|saved" gpurun_out/r04k_$k.log || true
done
