#!/bin/bash
# Round-2 closing evidence: smoke, GPU suite, the default bench (all lines, CPU baselines), kernel
# traces of every line in its own process, PMC passes of train / train88 / infer / blazeface.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r02b}
step() { echo "[$(date +%T)] $*"; }
step smoke
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
step tests
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/t_gpu.log; [ $rc = 0 ] || exit $rc
step bench
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
for line in train infer train88 blazeface p1 attn; do
  step "trace $line"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$line -o trace --output-format csv -- \
    python3 bench.py --only $line --no-cpu --steps 10 --warmup 2 > gpurun_out/prof_${TAG}_$line.log 2>&1 || exit $?
done
for line in train train88 infer blazeface; do
  LINE=$line TAG=$TAG bash scripts/pmc_r02.sh || exit $?
done
step done
