#!/bin/bash
# round-4: residual + spatial GPU tests, residual timing (+ phase stamps), attention bench line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_res.py tests/test_spatial.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04b_tests.log 2>&1 || { tail -30 gpurun_out/r04b_tests.log; exit 1; }
tail -2 gpurun_out/r04b_tests.log
timeout -k 10 200 python -u scripts/time_res.py 6 2>&1 | grep -v amdgpu.ids || exit 1
HPE_LIB=$PWD/varlibs/libhpe_rst.so timeout -k 10 200 python -u scripts/time_res.py 2 2>&1 | grep RSTAMP | tail -1 || exit 1
for t in 1 0; do
  HPE_ATTN_TAIL=$t timeout -k 10 300 python -u bench.py --only attn --no-cpu > gpurun_out/r04b_attn$t.json 2> gpurun_out/r04b_attn$t.err || { tail -5 gpurun_out/r04b_attn$t.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/r04b_attn$t.json').read().strip().splitlines()[-1])['attn']; print('attn tail=$t', round(d['ms_per_batch'],3), 'ms')"
done
