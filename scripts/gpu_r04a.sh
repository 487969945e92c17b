#!/bin/bash
# round-4 check: residual-stack tests (printed errors), the Model-88 complex trajectory test, the
# mlp2v race screen over many processes, and the P = 1 bench lines.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_drivers.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r04a_tests.log 2>&1 || { tail -30 gpurun_out/r04a_tests.log; exit 1; }
grep -E "passed|failed|max \|g" gpurun_out/r04a_tests.log | tail -12
timeout -k 10 400 python -u bench.py --only p1 --no-cpu > gpurun_out/r04a_p1.json 2> gpurun_out/r04a_p1.err || { tail -20 gpurun_out/r04a_p1.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open('gpurun_out/r04a_p1.json').read().strip().splitlines()[-1])
print({k: (round(v['us_per_step'], 2), v.get('fused')) for k, v in d['p1']['lines'].items() if isinstance(v, dict) and 'us_per_step' in v})
PY
PROCS=${PROCS:-40} R=${R:-250} TAG=r04a bash scripts/gpu_diag2.sh | sort | uniq -c
