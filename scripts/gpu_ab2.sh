#!/bin/bash
# A/B of libhpe variants (varlibs/libhpe_<v>.so; "base" = the in-tree library) on one bench line,
# interleaved ROUNDS times; then optionally the GPU test suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TAG=${TAG:-ab}
LINE=${LINE:-train}
for r in $(seq ${ROUNDS:-2}); do
  for v in base ${VARS}; do
    lib=""; [ "$v" != base ] && lib=$PWD/varlibs/libhpe_$v.so
    HPE_LIB=$lib timeout -k 10 300 python -u bench.py --only $LINE --no-cpu --steps ${STEPS:-20} --warmup 3 > gpurun_out/ab_${TAG}_${v}_$r.json 2> gpurun_out/ab_${TAG}_${v}_$r.err || exit $?
    python - "$v" "$LINE" gpurun_out/ab_${TAG}_${v}_$r.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
l = d if sys.argv[2] in ('train',) else d[sys.argv[2]]
print(sys.argv[1], {k: l.get(k) for k in ('ms_per_step', 'ms_per_batch')}, (l.get('roofline') or {}).get('frac'))
PY
  done
done
if [ "${TESTS:-0}" = 1 ]; then
  echo "[$(date +%T)] tests"
  timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_gpu_$TAG.log 2>&1
  rc=$?; tail -3 gpurun_out/t_gpu_$TAG.log; [ $rc = 0 ] || exit $rc
fi
echo "[$(date +%T)] done"
