#!/bin/bash
# round-4: mlp2v at 96x96 (multi-tile) vs the exact kernel in fresh processes, then inside a pytest
# process after the rest of the parity file
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for k in 1 2 3 4 5; do
  timeout -k 10 120 python -u scripts/diag_v.py 360 tanh 0.0 96 2 > gpurun_out/r04p_$k.log 2>&1 || { tail -5 gpurun_out/r04p_$k.log; exit 1; }
  grep "launch grid" gpurun_out/r04p_$k.log
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -k "8wave" --timeout 200 --timeout-method thread -s > gpurun_out/r04p_t1.log 2>&1; grep -E "^F=|passed|failed" gpurun_out/r04p_t1.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -k "8wave" --timeout 200 --timeout-method thread -s > gpurun_out/r04p_t2.log 2>&1; grep -E "^F=|passed|failed" gpurun_out/r04p_t2.log
