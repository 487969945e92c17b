#!/bin/bash
# round-4: BlazeFace stage kernel — GPU tests, per-op vs stage timing, kernel trace of the stage line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_blazeface.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04d_tests.log 2>&1 || { tail -30 gpurun_out/r04d_tests.log; exit 1; }
tail -2 gpurun_out/r04d_tests.log
HPE_BF_STAGE=0 timeout -k 10 300 python -u bench.py --only blazeface --no-cpu > gpurun_out/r04d_bf0.json 2> gpurun_out/r04d_bf0.err || { tail -20 gpurun_out/r04d_bf0.err; exit 1; }
timeout -k 10 300 python -u bench.py --only blazeface --no-cpu > gpurun_out/r04d_bf1.json 2> gpurun_out/r04d_bf1.err || { tail -20 gpurun_out/r04d_bf1.err; exit 1; }
python - <<'PY'
import json
for k in ('0', '1'):
    d = json.loads(open('gpurun_out/r04d_bf%s.json' % k).read().strip().splitlines()[-1])
    print('stage', k, json.dumps(d.get('blazeface'))[:600])
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04d_prof -o bf -- python3 -u bench.py --only blazeface --no-cpu > gpurun_out/r04d_prof.log 2>&1 || { tail -20 gpurun_out/r04d_prof.log; exit 1; }
find gpurun_out/r04d_prof -name '*kernel_stats.csv' | head -3
