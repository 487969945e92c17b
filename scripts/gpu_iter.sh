#!/bin/bash
# Iteration check on the GPU box (via gpurun): GPU parity suite, then a short bench.  BENCH_ARGS / PYTEST_K override.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/t_gpu.log 2>&1 && \
timeout -k 10 400 python -u bench.py --no-cpu ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
echo "rc=$rc"
tail -3 gpurun_out/t_gpu.log
grep -E "FAILED|Error|error" gpurun_out/t_gpu.log | head -20
cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
exit $rc
