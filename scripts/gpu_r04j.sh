#!/bin/bash
# round-4: BlazeFace per-kernel trace, per-op plan vs stage plan
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for st in 0 1; do
  HPE_BF_STAGE=$st timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04j_bf$st -o bf --output-format csv -- python3 -u bench.py --only blazeface --no-cpu --steps 10 --warmup 2 > gpurun_out/r04j_bf$st.log 2>&1 || { tail -20 gpurun_out/r04j_bf$st.log; exit 1; }
  f=$(find gpurun_out/r04j_bf$st -name '*kernel_stats.csv' | head -1)
  echo "== stage $st: $f"; cut -d, -f1-4 "$f" | head -14
done
