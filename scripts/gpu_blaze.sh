#!/bin/bash
# BlazeFace check on the GPU box (via gpurun): parity tests, timing, bench line, kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_blazeface.py tests/test_detector.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/tb.log 2>&1 && \
timeout -k 10 300 python -u scripts/time_blaze.py 1024 > gpurun_out/time_blaze.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_blaze -o run --output-format csv -- python3 scripts/time_blaze.py 1024 > gpurun_out/prof_blaze.log 2>&1
rc=$?
echo rc=$rc; tail -3 gpurun_out/tb.log; grep -E "FAILED|Error" gpurun_out/tb.log | head; cat gpurun_out/time_blaze.log; exit $rc
