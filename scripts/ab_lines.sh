#!/bin/bash
# A/B of bench lines between library builds on one GPU box (run via gpurun): the in-tree libhpe.so
# ("cur") and varlibs/libhpe_<name>.so for every name in LIBS, alternated REPS times so box drift
# hits both arms; ENVS adds arms of the in-tree library under one environment setting each
# ("HPE_X=0 HPE_Y=1": arm name = the setting).  Optional TESTS: a pytest -k expression run first.
# Prints one line per run: lib, line, ms per step / batch, roofline frac.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TAG=${TAG:-ab}
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu -k "$TESTS" --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc = 0 ] || exit $rc
fi
for r in $(seq 1 ${REPS:-2}); do
  for lib in cur $LIBS $ENVS; do
    unset HPE_LIB
    case "$lib" in
      cur) ;;
      *=*) export "$lib" ;;
      *) export HPE_LIB=$PWD/varlibs/libhpe_$lib.so ;;
    esac
    for l in ${LINES:-train}; do
      out=gpurun_out/${TAG}_${lib//=/-}_${l}_$r.json
      timeout -k 10 300 python -u bench.py --only $l --no-cpu ${BENCH_ARGS} > $out 2> ${out%.json}.err || { tail -5 ${out%.json}.err; exit 1; }
      python - "$lib" "$l" "$out" <<'PY'
import json, sys
lib, line, path = sys.argv[1:]
d = json.loads(open(path).read().strip().splitlines()[-1])
l = d if line == 'train' else d.get(line, d)
if line == 'p1':
    l = l.get('lines', l)
    print(lib, 'p1', {k: round(v['us_per_step'], 2) for k, v in l.items() if isinstance(v, dict) and 'us_per_step' in v})
else:
    rf = l.get('roofline') or {}
    print(lib, line, round(l.get('ms_per_step') or l.get('ms_per_batch'), 4), 'kernel_ms',
          round(rf.get('dominant_kernel_ms') or rf.get('kernel_ms') or 0, 4), 'frac', round(rf.get('frac') or 0, 4))
PY
    done
    case "$lib" in *=*) unset "${lib%%=*}" ;; esac
  done
done
unset HPE_LIB
