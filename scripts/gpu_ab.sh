#!/bin/bash
# A/B of mlp2 variant builds (varlibs/libhpe_<v>.so via HPE_LIB): train-line timing, phase stamps, split parity.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for v in ${VARIANTS}; do
  lib=$PWD/varlibs/libhpe_$v.so
  case $v in
    *s) HPE_LIB=$lib timeout -k 10 120 python -u bench.py --no-cpu --no-infer --no-blaze --no-train88 --steps 2 --warmup 1 > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err || exit 1
        grep STAMP gpurun_out/ab/$v.json | tail -2 ;;
    *)  HPE_LIB=$lib timeout -k 10 120 python -u bench.py --no-cpu --no-infer --no-blaze --no-train88 --steps 30 --warmup 3 > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err || exit 1
        echo "$v $(python -c "import json,sys; d=json.loads(open('gpurun_out/ab/$v.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['kernel_ms'])")"
        HPE_LIB=$lib timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread -k "split or sqnu665j" > gpurun_out/ab/$v.t.log 2>&1 || { echo "$v PARITY FAIL"; tail -20 gpurun_out/ab/$v.t.log; exit 1; }
        tail -1 gpurun_out/ab/$v.t.log ;;
  esac
done
