#!/bin/bash
# round-4: which mlp2v change moved the split gradient (test_train_step_8wave_kernel): current source
# with / without packed FP32, and the round-start source
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in ${VARS:-v1 v2 v3}; do
  HPE_LIB=$PWD/varlibs/libhpe_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -m gpu -k "test_train_step_8wave_kernel and tanh" --timeout 200 --timeout-method thread -s > gpurun_out/r04n_$v.log 2>&1
  echo "== $v: $(tail -1 gpurun_out/r04n_$v.log)"; grep -E "^F=|P=" gpurun_out/r04n_$v.log | head -12
done
