#!/bin/bash
# GPU suite + selected bench lines (LINES, default "p1 train88") with a one-line summary each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TAG=${TAG:-q}
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
  rc=$?; tail -3 gpurun_out/t_$TAG.log; [ $rc = 0 ] || exit $rc
fi
for l in ${LINES:-p1 train88}; do
  timeout -k 10 400 python -u bench.py --only $l --no-cpu > gpurun_out/${TAG}_$l.json 2> gpurun_out/${TAG}_$l.err || exit $?
  python - "$l" gpurun_out/${TAG}_$l.json <<'PY'
import json, sys
line = sys.argv[1]
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
l = d if line == 'train' else d.get(line, d)
if line == 'p1':
    l = l.get('lines', l)
    print('p1', {k: round(v['us_per_step'], 2) for k, v in l.items() if isinstance(v, dict) and 'us_per_step' in v})
else:
    print(line, l.get('ms_per_step') or l.get('ms_per_batch'), (l.get('roofline') or {}).get('frac'))
PY
done
