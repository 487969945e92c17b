set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -k "forward or golden or chain or spatial" > gpurun_out/t1.log 2>&1 && \
timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1
rc=$?; echo rc=$rc; tail -3 gpurun_out/t1.log; tail -c 2500 gpurun_out/bench.log; exit $rc
