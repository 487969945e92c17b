#!/bin/bash
# round-4: mlp2v without packed-FP32 VALU ops (the dropped product sits in a v_pk_fma_f32 lo half):
# per-process race screen and configs[3] timing against the current object
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in nopk base; do
  n=0
  for k in $(seq 1 8); do
    HPE_LIB=$PWD/varlibs/libhpe_$v.so HPE_SPLIT_ONLY=1 DIAG_SLEEP=0.01 timeout -k 10 120 python -u scripts/diag_repeat.py 4 30 sqnu665j 8 > gpurun_out/r04l_${v}_$k.log 2>&1 || { tail -5 gpurun_out/r04l_${v}_$k.log; exit 1; }
    d=$(grep -oE "[0-9]+ of [0-9]+ runs differ" gpurun_out/r04l_${v}_$k.log | cut -d' ' -f1); n=$((n + d))
  done
  echo "== $v: $n differing launches in 8 processes x 29"
done
for v in nopk base nopk base; do
  HPE_LIB=$PWD/varlibs/libhpe_$v.so timeout -k 10 200 python -u bench.py --only train --no-cpu > gpurun_out/r04l_train_$v.json 2> gpurun_out/r04l_train_$v.err || { tail -5 gpurun_out/r04l_train_$v.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r04l_train_$v.json').read().strip().splitlines()[-1]); print('$v', round(d['value']), d['ms_per_step'], d['roofline'].get('frac'))"
done
