#!/bin/bash
# Round-3 GPU pass: smoke, GPU suite, the default bench line, kernel traces of every bench line in
# its own process (summarised over the timed-region dispatches: scripts/summarize_profile.py), PMC
# passes.  Every GPU step has its own limit; the chain stops at the first failure.
#   TAG=r03a TESTS=1 BENCH=1 TRACE="train infer ..." PMC="train ..." bash scripts/gpu_r03.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r03}
STEPS=${STEPS:-10}
WARM=${WARM:-2}
step() { echo "[$(date +%T)] $*"; }
if [ "${SMOKE:-1}" = 1 ]; then
  step smoke
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
fi
if [ "${TESTS:-1}" = 1 ]; then
  step tests
  timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread ${TESTARGS:-} > gpurun_out/t_gpu_$TAG.log 2>&1
  rc=$?; tail -3 gpurun_out/t_gpu_$TAG.log; [ $rc = 0 ] || exit $rc
fi
if [ "${BENCH:-1}" = 1 ]; then
  step bench
  timeout -k 10 600 python -u bench.py ${BENCHARGS:-} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
  cat gpurun_out/bench_$TAG.json | head -c 600; echo
fi
for line in ${TRACE:-}; do
  step "trace $line"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$line -o trace --output-format csv -- \
    python3 bench.py --only $line --no-cpu --steps $STEPS --warmup $WARM > gpurun_out/prof_${TAG}_$line.log 2>&1 || exit $?
done
for line in ${PMC:-}; do
  LINE=$line TAG=$TAG bash scripts/pmc_r02.sh || exit $?
done
if [ -n "${EXTRA:-}" ]; then
  step "extra: $EXTRA"
  timeout -k 10 ${EXTRA_T:-600} bash -c "$EXTRA" > gpurun_out/extra_$TAG.log 2>&1 || exit $?
fi
step done
