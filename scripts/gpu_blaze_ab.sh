#!/bin/bash
# A/B timing of BlazeFace planner variants (via gpurun) + per-kernel trace of the default variant
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_blazeface.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tb.log 2>&1 && \
HPE_BF_NORECOMPUTE=0 timeout -k 10 300 python -u scripts/time_blaze.py 1024 > gpurun_out/time_a.log 2>&1 && \
HPE_BF_NORECOMPUTE=1 timeout -k 10 300 python -u scripts/time_blaze.py 1024 > gpurun_out/time_b.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_blaze -o run --output-format csv -- python3 scripts/time_blaze.py 1024 > gpurun_out/prof_blaze.log 2>&1
rc=$?
echo rc=$rc; tail -2 gpurun_out/tb.log; echo A; cat gpurun_out/time_a.log | tail -1; echo B; cat gpurun_out/time_b.log | tail -1; exit $rc
