#!/bin/bash
# round-4: A1 park rows on distinct bank quads (a1_row) — all GPU tests, configs[3] train A/B against
# the previous big object (varlibs/libhpe_old.so), LDS PMC pass; phase stamps of the P = 1 per-step kernel
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04s_tests.log 2>&1 || { tail -30 gpurun_out/r04s_tests.log; exit 1; }
tail -2 gpurun_out/r04s_tests.log
for k in new old new old; do
  if [ $k = old ]; then L=$PWD/varlibs/libhpe_old.so; else L=; fi
  HPE_LIB=$L timeout -k 10 300 python -u bench.py --only train --no-cpu > gpurun_out/r04s_train_$k.json 2> gpurun_out/r04s_train_$k.err || { tail -20 gpurun_out/r04s_train_$k.err; exit 1; }
  python - $k <<'PY'
import json, sys
d = json.loads(open('gpurun_out/r04s_train_%s.json' % sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d['value'], d['ms_per_step'], d['roofline']['frac'])
PY
done
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -d gpurun_out/pmc_r04s_train -o pmc --output-format csv -- python3 bench.py --only train --no-cpu --steps 5 --warmup 1 > gpurun_out/pmc_r04s_train.log 2>&1 || { tail -20 gpurun_out/pmc_r04s_train.log; exit 1; }
for bs in 128 512; do
  HPE_LIB=$PWD/varlibs/libhpe_stamps.so timeout -k 10 200 python -u scripts/p1_stamps.py $bs > gpurun_out/r04s_stamps_$bs.log 2>&1 || { tail -20 gpurun_out/r04s_stamps_$bs.log; exit 1; }
  python - $bs <<'PY'
import re, sys, numpy as np
L = open('gpurun_out/r04s_stamps_%s.log' % sys.argv[1]).read().splitlines()
for w in ('w0', 'w5'):
    rows = [list(map(int, re.findall(r' (\d+)', l.split(w, 1)[1]))) for l in L if l.startswith('STAMP ' + w)]
    if rows:
        print(sys.argv[1], w, len(rows), 'pro bwd+tail bar1 stage fwdmfma act+part bar2 head bar3 presplit', np.median(np.array(rows)[len(rows) // 2:], 0).astype(int).tolist())
e = [list(map(int, re.findall(r' (\d+)', l))) for l in L if l.startswith('STAMPEND')]
if e:
    print(sys.argv[1], 'end', len(e), 'flush total real(100MHz)', np.median(np.array(e)[len(e) // 2:], 0).astype(int).tolist())
PY
done
echo done
