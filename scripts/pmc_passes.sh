#!/bin/bash
# PMC passes over one command (each pass its own rocprofv3 run, kernel-trace only, hard time limit):
#   PASSES="CTR CTR ...;CTR ..." (';'-separated passes), TAG names the output dirs under gpurun_out/.
#   usage: PASSES=... TAG=x scripts/pmc_passes.sh python3 scripts/time_blaze.py 256
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
IFS=';' read -ra PS <<< "$PASSES"
for P in "${PS[@]}"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace -d gpurun_out/pmc_${TAG}_$i -o pmc --output-format csv -- "$@" > gpurun_out/pmc_${TAG}_$i.log 2>&1 || { echo "pass $i ($P) failed"; tail -5 gpurun_out/pmc_${TAG}_$i.log; exit 1; }
done
echo done
