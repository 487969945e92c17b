#!/bin/bash
# Full GPU parity suite + smoke at HEAD (run via gpurun).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_full.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?
echo "rc=$rc"
tail -3 gpurun_out/t_full.log
cat gpurun_out/smoke.log
exit $rc
