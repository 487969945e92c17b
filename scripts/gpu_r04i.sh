#!/bin/bash
# round-4: mlp2v race screen per process (the differing launches come in a process's first few):
# K processes x R launches each, idle gaps between launches, base vs no-SLP object
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in ${VARS:-base noslp}; do
  for k in $(seq 1 ${K:-8}); do
    HPE_LIB=$PWD/varlibs/libhpe_$v.so HPE_SPLIT_ONLY=1 DIAG_SLEEP=${SLEEP:-0.01} timeout -k 10 120 python -u scripts/diag_repeat.py 4 ${R:-40} sqnu665j 8 > gpurun_out/r04i_${v}_$k.log 2>&1 || { tail -5 gpurun_out/r04i_${v}_$k.log; exit 1; }
    echo "== $v $k: $(grep -E 'runs differ' gpurun_out/r04i_${v}_$k.log)"; grep -E "^run" gpurun_out/r04i_${v}_$k.log | head -2 | cut -c1-400
  done
done
