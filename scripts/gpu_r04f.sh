#!/bin/bash
# round-4: mlp2v race screen at sqnu665j 8x8 maps, 4 images (one tile per workgroup): A/B variants
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in base bargme waitgme barflush; do
  HPE_LIB=$PWD/varlibs/libhpe_$v.so HPE_SPLIT_ONLY=1 timeout -k 10 200 python -u scripts/diag_repeat.py 4 ${R:-600} sqnu665j 8 > gpurun_out/r04f_$v.log 2>&1 || { tail -5 gpurun_out/r04f_$v.log; exit 1; }
  echo "== $v"; grep -E "runs differ|guard fired" gpurun_out/r04f_$v.log; grep -E "^run" gpurun_out/r04f_$v.log | head -3
done
