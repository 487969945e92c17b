#!/bin/bash
# Round evidence after the fp16-split GEMMs: new parity tests, full bench (CPU baselines), kernel trace,
# FETCH_SIZE / WRITE_SIZE passes (separate runs, kernel-trace only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -s -m gpu --timeout 120 --timeout-method thread -k "split" > gpurun_out/t_split.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o trace --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/prof_trace.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/prof_fetch -o fetch --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/prof_write -o write --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_write.log 2>&1
rc=$?
echo "rc=$rc"
grep -E "max \||passed|failed" gpurun_out/t_split.log | tail -8
cat gpurun_out/bench.json
exit $rc
