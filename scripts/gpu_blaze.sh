set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_blazeface.py tests/test_detector.py -x -q > gpurun_out/tb.log 2>&1 && \
timeout -k 10 300 python scripts/time_blaze.py 1024 > gpurun_out/time_blaze.log 2>&1 && timeout -k 10 400 python bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/bench_blaze.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_blaze -o run -- python $GRAFT_REPO_ROOT/scripts/time_blaze.py 1024 > $GRAFT_REPO_ROOT/gpurun_out/prof_blaze.log 2>&1
rc=$?; cd $GRAFT_REPO_ROOT; echo rc=$rc; tail -5 gpurun_out/tb.log; cat gpurun_out/time_blaze.log; exit $rc
