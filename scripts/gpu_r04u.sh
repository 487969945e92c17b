#!/bin/bash
# round-4: A1 padding restricted to the 12-wave kernel (the 4-wave one keeps its 4 workgroups per CU)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04u_tests.log 2>&1 || { tail -30 gpurun_out/r04u_tests.log; exit 1; }
tail -2 gpurun_out/r04u_tests.log
for line in train88 train; do
  timeout -k 10 300 python -u bench.py --only $line --no-cpu > gpurun_out/r04u_$line.json 2> gpurun_out/r04u_$line.err || { tail -20 gpurun_out/r04u_$line.err; exit 1; }
  python - $line <<'PY'
import json, sys
d = json.loads(open('gpurun_out/r04u_%s.json' % sys.argv[1]).read().strip().splitlines()[-1])
v = d if sys.argv[1] == 'train' else d[sys.argv[1]]
print(sys.argv[1], v['value'], v.get('ms_per_step'), v['roofline']['frac'], v['roofline'].get('kernel'))
PY
done
echo done
