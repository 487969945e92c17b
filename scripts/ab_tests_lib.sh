#!/bin/bash
# Run a pytest -k selection of the GPU tests against varlibs/libhpe_<name>.so (HPE_LIB) for each
# name in LIBS, then the A/B bench lines (scripts/ab_lines.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for lib in $LIBS; do
  HPE_LIB=$PWD/varlibs/libhpe_$lib.so timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu -k "$TESTS" --timeout 300 --timeout-method thread > gpurun_out/abt_$lib.log 2>&1
  rc=$?; echo "$lib tests rc=$rc $(tail -1 gpurun_out/abt_$lib.log)"; [ $rc = 0 ] || exit $rc
done
TESTS= scripts/ab_lines.sh
