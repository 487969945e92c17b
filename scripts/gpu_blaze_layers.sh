#!/bin/bash
# BlazeFace per-layer evidence (run via gpurun): kernel traces of scripts/time_blaze.py with the
# staged plan (default) and the per-op plan (HPE_BF_STAGE=0 HPE_BF_FRONT=0), then FETCH_SIZE / WRITE_SIZE passes
# of the staged plan (separate runs, kernel-trace only).  Summarise locally with
# scripts/blaze_layers.py (one per trace) and scripts/pmc_quick.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05}
B=${BATCH:-1024}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_blaze -o run --output-format csv -- \
  python3 scripts/time_blaze.py $B > gpurun_out/prof_${TAG}_blaze.log 2>&1 || exit $?
HPE_BF_STAGE=0 HPE_BF_FRONT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_blaze_perop -o run \
  --output-format csv -- python3 scripts/time_blaze.py $B > gpurun_out/prof_${TAG}_blaze_perop.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/pmc_${TAG}_blaze_$c -o pmc --output-format csv -- \
    python3 scripts/time_blaze.py $B > gpurun_out/pmc_${TAG}_blaze_$c.log 2>&1 || exit $?
done
grep -h "img/s" gpurun_out/prof_${TAG}_blaze.log gpurun_out/prof_${TAG}_blaze_perop.log
