#!/bin/bash
# GPU suite + selected bench lines (A/B of an env switch via AB_ENV="NAME=a NAME=b").
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { echo "[$(date +%T)] $*"; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step tests
  timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/t_gpu.log 2>&1
  rc=$?; tail -3 gpurun_out/t_gpu.log; [ $rc = 0 ] || exit $rc
fi
i=0
for e in ${AB_ENV:-NONE=1}; do
  i=$((i+1))
  step "bench $e"
  env $e timeout -k 10 300 python -u bench.py --only ${LINES:-train} --no-cpu --steps ${STEPS:-20} --warmup 3 > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err || exit $?
  python -c "
import json,sys; d=json.loads(open('gpurun_out/ab_$i.json').read().strip().splitlines()[-1])
for k,v in d.items():
    if isinstance(v, dict) and 'value' in v: print('$e', k, round(v['value']), v.get('ms_per_step', v.get('ms_per_batch')), (v.get('roofline') or {}).get('frac'))
if 'value' in d: print('$e', 'train', round(d['value']), d['ms_per_step'], d['roofline']['frac'])
"
done
step done
