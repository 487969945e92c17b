#!/bin/bash
# round-4: mlp2_kernel A1 park on distinct bank quads + one-batch prologue — all GPU tests, configs[3]
# train and P = 1 lines A/B against the previous mlp2 objects (varlibs/libhpe_old.so), prologue stamps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if ! timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04t_tests.log 2>&1; then
  rc=$?; tail -30 gpurun_out/r04t_tests.log; [ $rc -ne 1 ] && exit 1
  # test failure (not a fault / timeout): the A1-only build (varlibs/libhpe_a1.so) through the same suite
  HPE_LIB=$PWD/varlibs/libhpe_a1.so timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04t_tests_a1.log 2>&1; echo "a1 rc=$?"; tail -3 gpurun_out/r04t_tests_a1.log; exit 1
fi
tail -2 gpurun_out/r04t_tests.log
for k in new old new old; do
  if [ $k = old ]; then L=$PWD/varlibs/libhpe_old.so; else L=; fi
  HPE_LIB=$L timeout -k 10 300 python -u bench.py --only train --no-cpu > gpurun_out/r04t_train_$k.json 2> gpurun_out/r04t_train_$k.err || { tail -20 gpurun_out/r04t_train_$k.err; exit 1; }
  python - $k <<'PY'
import json, sys
d = json.loads(open('gpurun_out/r04t_train_%s.json' % sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['frac'])
PY
done
for k in new old; do
  if [ $k = old ]; then L=$PWD/varlibs/libhpe_old.so; else L=; fi
  HPE_LIB=$L timeout -k 10 400 python -u bench.py --only p1 --no-cpu > gpurun_out/r04t_p1_$k.json 2> gpurun_out/r04t_p1_$k.err || { tail -20 gpurun_out/r04t_p1_$k.err; exit 1; }
  python - $k <<'PY'
import json, sys
d = json.loads(open('gpurun_out/r04t_p1_%s.json' % sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], {k: round(v['us_per_step'], 2) for k, v in d['p1']['lines'].items() if isinstance(v, dict) and 'us_per_step' in v})
PY
done
HPE_LIB=$PWD/varlibs/libhpe_stamps.so timeout -k 10 200 python -u scripts/p1_stamps.py 128 > gpurun_out/r04t_stamps_128.log 2>&1 || { tail -20 gpurun_out/r04t_stamps_128.log; exit 1; }
python - <<'PY'
import re, numpy as np
L = open('gpurun_out/r04t_stamps_128.log').read().splitlines()
for w in ('w0', 'w5'):
    rows = [list(map(int, re.findall(r' (\d+)', l.split(w, 1)[1]))) for l in L if l.startswith('STAMP ' + w)]
    if rows:
        print(w, len(rows), 'pro bwd+tail bar1 stage fwdmfma act+part bar2 head bar3 presplit', np.median(np.array(rows)[len(rows) // 2:], 0).astype(int).tolist())
PY
echo done
