set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_h5io.py tests/test_features.py tests/test_sweep.py -x -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_new.log 2>&1
rc=$?; tail -15 gpurun_out/t_new.log; exit $rc
