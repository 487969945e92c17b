#!/bin/bash
# mlp2v_kernel check: targeted parity tests, the headline line with and without it (A/B), stamps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TAG=${TAG:-v1}
if [ "${TESTS:-1}" = 1 ]; then
  echo "[$(date +%T)] tests"
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu --timeout 120 --timeout-method thread -k "${K:-8wave or split_vs_exact or wide_dropout}" -s > gpurun_out/t_$TAG.log 2>&1
  rc=$?; grep -E "PASS|FAIL|Error|error|float64" gpurun_out/t_$TAG.log | tail -30; [ $rc = 0 ] || exit $rc
fi
for v in ${VS:-1 0}; do
  echo "[$(date +%T)] bench V=$v"
  HPE_MLP2_V=$v timeout -k 10 300 python -u bench.py --only ${LINE:-train} --no-cpu --steps 20 --warmup 3 > gpurun_out/b_${TAG}_$v.json 2> gpurun_out/b_${TAG}_$v.err || exit $?
  python -c "import json;d=json.loads(open('gpurun_out/b_${TAG}_$v.json').read().strip().splitlines()[-1]);print('V=$v', d['ms_per_step'], d['roofline']['frac'])"
done
if [ -f varlibs/libhpe_stamps.so ] && [ "${STAMPS:-1}" = 1 ]; then
  echo "[$(date +%T)] stamps"
  HPE_LIB=$PWD/varlibs/libhpe_stamps.so timeout -k 10 200 python -u bench.py --only train --no-cpu --steps 2 --warmup 1 > gpurun_out/stamps_$TAG.log 2>&1 || exit $?
  grep STAMP gpurun_out/stamps_$TAG.log | tail -2
fi
if [ -n "${PROF:-}" ]; then
  echo "[$(date +%T)] trace"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o trace --output-format csv -- python3 bench.py --only train --no-cpu --steps 10 --warmup 2 > gpurun_out/prof_$TAG.log 2>&1 || exit $?
fi
echo "[$(date +%T)] done"
