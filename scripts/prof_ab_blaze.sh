#!/bin/bash
# rocprofv3 kernel-trace stats of scripts/time_blaze.py for the in-tree lib and varlibs/libhpe_<name>.so (LIBS)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in cur $LIBS; do
  if [ $lib = cur ]; then unset HPE_LIB; else export HPE_LIB=$PWD/varlibs/libhpe_$lib.so; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/pab_$lib -o run --output-format csv -- python3 -u scripts/time_blaze.py 1024 > gpurun_out/pab_$lib.log 2>&1 || exit 1
done
