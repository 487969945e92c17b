#!/bin/bash
# Round check on the GPU box (run via gpurun): smoke, GPU parity suite, bench (all lines), and a
# rocprofv3 kernel trace of each bench line in its own process (profiles keyed per line), at the
# bench's default step counts, so a traced line's JSON and its trace come from one run.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r06}
SKIP_TESTS=${SKIP_TESTS:-0}
step() { echo "[$(date +%T)] $*"; }
if [ "${SMOKE:-1}" = 1 ]; then
  step smoke
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
fi
if [ "$SKIP_TESTS" != 1 ]; then
  step tests
  timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/t_gpu.log 2>&1
  rc=$?; tail -3 gpurun_out/t_gpu.log; [ $rc = 0 ] || exit $rc
fi
if [ "${BENCH:-1}" = 1 ]; then
  step bench
  timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
  cat gpurun_out/bench_$TAG.json
fi
if [ "${PROFILE:-1}" = 1 ]; then
  for line in ${LINES:-train infer train88 blazeface blazeface_b1 p1 attn}; do
    step "trace $line"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$line -o trace --output-format csv -- \
      python3 bench.py --only $line --no-cpu --steps ${TRACE_STEPS:-20} --warmup ${TRACE_WARMUP:-3} > gpurun_out/prof_${TAG}_$line.log 2>&1 || exit $?
  done
fi
if [ "${PMC:-1}" = 1 ]; then
  for line in ${PMC_LINES:-train train88 infer blazeface}; do
    TAG=$TAG LINE=$line scripts/pmc_line.sh || exit $?
  done
fi
step done
