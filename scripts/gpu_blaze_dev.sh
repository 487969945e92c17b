#!/bin/bash
# BlazeFace development loop on the GPU box: the BlazeFace GPU tests, timing at 1024 / 8 / 1 frames,
# and (if varlibs/libhpe_bfs.so exists) the stage kernel's per-op stamps of workgroup 0.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
TAG=${TAG:-bd}
timeout -k 10 400 python -u -m pytest tests/test_blazeface.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/${TAG}_t.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_t.log; [ $rc = 0 ] || exit $rc
for n in 1024 8 1; do
  timeout -k 10 120 python -u scripts/time_blaze.py $n 2>/dev/null | tee -a gpurun_out/${TAG}_time.log || exit 1
done
if [ -f varlibs/libhpe_bfs.so ]; then
  HPE_LIB=$PWD/varlibs/libhpe_bfs.so timeout -k 10 200 python -u scripts/time_blaze.py 1024 > gpurun_out/${TAG}_bfs.log 2>&1 || exit 1
fi
