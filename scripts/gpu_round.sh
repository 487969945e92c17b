#!/bin/bash
# Full round check on the GPU box (run via gpurun): smoke, GPU parity suite, bench, rocprof kernel trace.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r01}
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_gpu.log 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --no-cpu --steps 10 --warmup 2 > gpurun_out/prof_$TAG.log 2>&1
rc=$?
echo "rc=$rc"
tail -3 gpurun_out/t_gpu.log
cat gpurun_out/bench.json
exit $rc
