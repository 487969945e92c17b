#!/bin/bash
# round-4: padded A1 park rows + component-major loss accumulators in mlp2_kernel — all GPU tests,
# configs[3] train A/B against the previous big object (varlibs/libhpe_old.so), LDS PMC pass
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04r_tests.log 2>&1 || { tail -30 gpurun_out/r04r_tests.log; exit 1; }
tail -2 gpurun_out/r04r_tests.log
for k in new old new old; do
  if [ $k = old ]; then L=$PWD/varlibs/libhpe_old.so; else L=; fi
  HPE_LIB=$L timeout -k 10 300 python -u bench.py --only train --no-cpu > gpurun_out/r04r_train_$k.json 2> gpurun_out/r04r_train_$k.err || { tail -20 gpurun_out/r04r_train_$k.err; exit 1; }
  python - $k <<'PY'
import json, sys
d = json.loads(open('gpurun_out/r04r_train_%s.json' % sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], d['value'], d['ms_per_step'], json.dumps(d.get('roofline'))[:200])
PY
done
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -d gpurun_out/pmc_r04r_train -o pmc --output-format csv -- python3 bench.py --only train --no-cpu --steps 5 --warmup 1 > gpurun_out/pmc_r04r_train.log 2>&1 || { tail -20 gpurun_out/pmc_r04r_train.log; exit 1; }
echo done
