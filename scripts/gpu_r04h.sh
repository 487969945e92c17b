#!/bin/bash
# round-4: mlp2v race screen + train-line timing, base vs no-SLP object; then the r04g measurements
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in noslp base; do
  HPE_LIB=$PWD/varlibs/libhpe_$v.so HPE_SPLIT_ONLY=1 timeout -k 10 200 python -u scripts/diag_repeat.py 4 600 sqnu665j 8 > gpurun_out/r04h_$v.log 2>&1 || { tail -5 gpurun_out/r04h_$v.log; exit 1; }
  echo "== $v"; grep -E "runs differ" gpurun_out/r04h_$v.log; grep -E "^run" gpurun_out/r04h_$v.log | head -3
done
for v in noslp base noslp base; do
  HPE_LIB=$PWD/varlibs/libhpe_$v.so timeout -k 10 200 python -u bench.py --only train --no-cpu > gpurun_out/r04h_train_$v.json 2> gpurun_out/r04h_train_$v.err || { tail -5 gpurun_out/r04h_train_$v.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r04h_train_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['roofline'].get('frac'), d['roofline'].get('kernel_ms'))"
done
bash scripts/gpu_r04g.sh
