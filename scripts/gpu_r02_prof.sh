#!/bin/bash
# Round-2 evidence pass on the GPU box: kernel traces of every bench line (own process each), the
# PMC passes of the train / train88 / infer lines, and the Model-96 seed-spread run.  Every GPU
# step has its own limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r02}
step() { echo "[$(date +%T)] $*"; }
for line in ${LINES:-train infer train88 blazeface p1}; do
  step "trace $line"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$line -o trace --output-format csv -- \
    python3 bench.py --only $line --no-cpu --steps 10 --warmup 2 > gpurun_out/prof_${TAG}_$line.log 2>&1 || exit $?
done
for line in ${PMC_LINES:-train train88 infer}; do
  LINE=$line TAG=$TAG bash scripts/pmc_r02.sh || exit $?
done
if [ "${SEEDS:-0}" != 0 ]; then
  step "seed spread"
  timeout -k 10 600 python3 -u scripts/seed_spread_96.py $SEEDS > gpurun_out/seed_spread.log 2>&1 || exit $?
fi
for line in ${LATE_LINES:-attn}; do
  step "trace $line"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_$line -o trace --output-format csv -- \
    python3 bench.py --only $line --no-cpu --steps 10 --warmup 2 > gpurun_out/prof_${TAG}_$line.log 2>&1 || exit $?
done
step done
