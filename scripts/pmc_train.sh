#!/bin/bash
# PMC passes over the configs[3] training line only: split (default) vs exact-fp32 kernels
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS"
B="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
ARGS="--steps 3 --warmup 1 --no-cpu --no-infer --no-blaze --no-train88"
timeout -k 10 120 rocprofv3 --pmc $A --kernel-trace -d gpurun_out/pmc_s_a -o p --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc1.log 2>&1 && \
timeout -k 10 120 rocprofv3 --pmc $B --kernel-trace -d gpurun_out/pmc_s_b -o p --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc2.log 2>&1 && \
HPE_EXACT_FP32=1 timeout -k 10 120 rocprofv3 --pmc $A --kernel-trace -d gpurun_out/pmc_e_a -o p --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc3.log 2>&1 && \
HPE_EXACT_FP32=1 timeout -k 10 120 rocprofv3 --pmc $B --kernel-trace -d gpurun_out/pmc_e_b -o p --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc4.log 2>&1
rc=$?
echo "rc=$rc"
exit $rc
