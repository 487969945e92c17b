#!/bin/bash
# targeted parity tests of the in-tree library, A/B against variant libraries, stamps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TAG=${TAG:-pipe}
echo "[$(date +%T)] tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "${K:-8wave or split_vs_exact or wide_dropout}" > gpurun_out/t_$TAG.log 2>&1
rc=$?; tail -2 gpurun_out/t_$TAG.log; [ $rc = 0 ] || exit $rc
TESTS=0 TAG=$TAG VARS="$VARS" ROUNDS=${ROUNDS:-2} bash scripts/gpu_ab2.sh || exit $?
if [ -f varlibs/libhpe_stamps.so ]; then
  HPE_LIB=$PWD/varlibs/libhpe_stamps.so timeout -k 10 200 python -u bench.py --only train --no-cpu --steps 2 --warmup 1 > gpurun_out/stamps_$TAG.log 2>&1 || exit $?
  grep STAMP gpurun_out/stamps_$TAG.log | tail -2
fi
