#!/bin/bash
# Race screen of the headline training kernel (scripts/diag_repeat.py) with the guard diagnostics:
# default schedule, then the split kernel alone (HPE_SPLIT_ONLY=1).  RUNS: "n:R ..." pairs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TAG=${TAG:-d}
for nr in ${RUNS:-2:300 24:60}; do
  n=${nr%%:*}; r=${nr##*:}
  timeout -k 10 300 python -u scripts/diag_repeat.py $n $r > gpurun_out/${TAG}_n${n}.log 2>&1 || { tail -5 gpurun_out/${TAG}_n${n}.log; exit 1; }
  grep -E "guard fired in|runs differ" gpurun_out/${TAG}_n${n}.log
  HPE_SPLIT_ONLY=1 timeout -k 10 300 python -u scripts/diag_repeat.py $n $r > gpurun_out/${TAG}_so_n${n}.log 2>&1 || { tail -5 gpurun_out/${TAG}_so_n${n}.log; exit 1; }
  grep -E "guard fired in|runs differ" gpurun_out/${TAG}_so_n${n}.log
done
