#!/bin/bash
# BlazeFace forward A/B between the in-tree library and varlibs/libhpe_<name>.so (LIBS), REPS
# alternations, 1024 frames (N) per call; optional bit-identity check of each variant (TESTS=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for r in $(seq 1 ${REPS:-2}); do
  for lib in cur $LIBS; do
    if [ $lib = cur ]; then unset HPE_LIB; else export HPE_LIB=$PWD/varlibs/libhpe_$lib.so; fi
    echo -n "$lib "; timeout -k 10 120 python -u scripts/time_blaze.py ${N:-1024} 2>/dev/null || exit 1
  done
done
unset HPE_LIB
if [ "${TESTS:-0}" = 1 ]; then
  for lib in cur $LIBS; do
    if [ $lib = cur ]; then unset HPE_LIB; else export HPE_LIB=$PWD/varlibs/libhpe_$lib.so; fi
    timeout -k 10 300 python -u -m pytest tests/test_blazeface.py -x -q -m gpu -k "bit_for_bit" --timeout 120 > gpurun_out/abb_$lib.log 2>&1
    echo "$lib tests rc=$? $(tail -1 gpurun_out/abb_$lib.log)"
  done
fi
