#!/bin/bash
# round-4: residual timing + stamps, P = 1 lines, BlazeFace stage tests + timing + trace, train line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/time_res.py 6 2>&1 | grep -v amdgpu.ids || exit 1
HPE_LIB=$PWD/varlibs/libhpe_rst.so timeout -k 10 200 python -u scripts/time_res.py 2 2>&1 | grep RSTAMP | tail -1 || exit 1
timeout -k 10 400 python -u bench.py --only p1 --no-cpu > gpurun_out/r04c_p1.json 2> gpurun_out/r04c_p1.err || { tail -20 gpurun_out/r04c_p1.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open('gpurun_out/r04c_p1.json').read().strip().splitlines()[-1])
print({k: (round(v['us_per_step'], 2), v.get('fused')) for k, v in d['p1']['lines'].items() if isinstance(v, dict) and 'us_per_step' in v})
PY
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
timeout -k 10 300 python -u bench.py --only train --no-cpu > gpurun_out/r04c_train.json 2> gpurun_out/r04c_train.err || { tail -20 gpurun_out/r04c_train.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open('gpurun_out/r04c_train.json').read().strip().splitlines()[-1])
print('train', d['value'], d['ms_per_step'], json.dumps(d.get('roofline'))[:400])
PY
