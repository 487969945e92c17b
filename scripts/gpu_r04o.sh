#!/bin/bash
# round-4: where mlp2v departs from the 12-wave / exact kernels (1 tile per workgroup, dropout)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
i=0
for cfg in "360 tanh 0.3 8 40" "360 tanh 0.3 8 40" "360 tanh 0.0 8 40" "200 elu 0.2 8 40" "360 tanh 0.3 96 2"; do
  i=$((i+1))
  timeout -k 10 120 python -u scripts/diag_v.py $cfg > gpurun_out/r04o_$i.log 2>&1 || { tail -5 gpurun_out/r04o_$i.log; exit 1; }
  echo "== $cfg"; grep -v amdgpu.ids gpurun_out/r04o_$i.log
done
