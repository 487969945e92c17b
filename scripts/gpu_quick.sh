#!/bin/bash
# quick GPU check: smoke + a subset of parity tests (run via gpurun)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -k "${K:-hrchr82r or sqnu665j or spatial or evaluate}" > gpurun_out/t1.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
