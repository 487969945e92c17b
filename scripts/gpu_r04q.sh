#!/bin/bash
# round-4: BlazeFace stage (fields hoisted) tests + trace; 12-wave head patch: parity subset + train line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_blazeface.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04q_bf_tests.log 2>&1 || { tail -30 gpurun_out/r04q_bf_tests.log; exit 1; }
tail -1 gpurun_out/r04q_bf_tests.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "8wave or repeatable or split_vs_exact or trajectory or fit_steps" --timeout 300 --timeout-method thread > gpurun_out/r04q_par.log 2>&1 || { tail -30 gpurun_out/r04q_par.log; exit 1; }
tail -1 gpurun_out/r04q_par.log
timeout -k 10 300 python -u bench.py --only train --no-cpu > gpurun_out/r04q_train.json 2> gpurun_out/r04q_train.err || { tail -20 gpurun_out/r04q_train.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r04q_train.json').read().strip().splitlines()[-1]); print('train', round(d['value']), d['ms_per_step'], d['roofline'].get('frac'))"
HPE_BF_STAGE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04q_bf1 -o bf --output-format csv -- python3 -u bench.py --only blazeface --no-cpu --steps 10 --warmup 2 > gpurun_out/r04q_bf1.log 2>&1 || { tail -20 gpurun_out/r04q_bf1.log; exit 1; }
f=$(find gpurun_out/r04q_bf1 -name '*kernel_stats.csv' | head -1); cut -d, -f1-4 "$f" | head -8
python -c "import json; d=json.loads(open('gpurun_out/r04q_bf1.log').read().strip().splitlines()[-1]) if False else None" || true
grep -o '"blazeface": {[^}]*' gpurun_out/r04q_bf1.log | head -c 400
