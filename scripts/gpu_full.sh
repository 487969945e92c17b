#!/bin/bash
# GPU parity (fused + generic paths) then bench (run via gpurun)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > gpurun_out/t_fused.log 2>&1 && \
HPE_FUSED=0 timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -k "sqnu665j or 0g73t16n or stoqa9pt or spatial" > gpurun_out/t_generic.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
