#!/bin/bash
# round-4: A1 park padding in the 4-wave mlp2_kernel too (3-float loss accumulators keep its LDS) —
# all GPU tests, Model-88 train A/B against the previous library (varlibs/libhpe_prev.so), configs[3] train
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04v_tests.log 2>&1 || { tail -30 gpurun_out/r04v_tests.log; exit 1; }
tail -2 gpurun_out/r04v_tests.log
for k in new prev new prev; do
  if [ $k = prev ]; then L=$PWD/varlibs/libhpe_prev.so; else L=; fi
  HPE_LIB=$L timeout -k 10 300 python -u bench.py --only train88 --no-cpu > gpurun_out/r04v_$k.json 2> gpurun_out/r04v_$k.err || { tail -20 gpurun_out/r04v_$k.err; exit 1; }
  python - $k <<'PY'
import json, sys
d = json.loads(open('gpurun_out/r04v_%s.json' % sys.argv[1]).read().strip().splitlines()[-1])['train88']
print(sys.argv[1], d['value'], d.get('ms_per_step'), d['roofline']['frac'])
PY
done
timeout -k 10 300 python -u bench.py --only train --no-cpu > gpurun_out/r04v_train.json 2> gpurun_out/r04v_train.err || { tail -20 gpurun_out/r04v_train.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r04v_train.json').read().strip().splitlines()[-1]); print('train', d['value'], d['ms_per_step'])"
echo done
