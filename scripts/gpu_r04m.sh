#!/bin/bash
# round-4: parity suite (C step loop, no-packed mlp2 object), P = 1 lines, train line, BlazeFace trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04m_tests.log 2>&1 || { tail -40 gpurun_out/r04m_tests.log; exit 1; }
tail -2 gpurun_out/r04m_tests.log
timeout -k 10 400 python -u bench.py --only p1 --no-cpu > gpurun_out/r04m_p1.json 2> gpurun_out/r04m_p1.err || { tail -20 gpurun_out/r04m_p1.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open('gpurun_out/r04m_p1.json').read().strip().splitlines()[-1])
print({k: (round(v['us_per_step'], 2), v.get('fused')) for k, v in d['p1']['lines'].items() if isinstance(v, dict) and 'us_per_step' in v})
PY
timeout -k 10 300 python -u bench.py --only train --no-cpu > gpurun_out/r04m_train.json 2> gpurun_out/r04m_train.err || { tail -20 gpurun_out/r04m_train.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r04m_train.json').read().strip().splitlines()[-1]); print('train', round(d['value']), d['ms_per_step'], d['roofline'].get('frac'))"
bash scripts/gpu_r04j.sh
