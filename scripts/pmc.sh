#!/bin/bash
# one rocprofv3 PMC pass (counters in $PMC) over a short bench run
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --pmc $PMC --kernel-trace -d gpurun_out/prof_pmc -o pmc --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu ${BENCH_ARGS} > gpurun_out/prof_pmc.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
