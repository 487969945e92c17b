#!/bin/bash
# PMC passes (one rocprofv3 run per counter group, never combined with tracing domains) of one bench
# line, per MI355X_MICROARCH.md §rocprofv3 PMC slots: <= 8 SQ, <= 4 TCC (FETCH_SIZE 3, WRITE_SIZE 2),
# <= 2 GRBM per pass.  Output: gpurun_out/pmc_<tag>_<line>_<pass>/
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r05}
LINE=${LINE:-train}
ARGS="--only $LINE --no-cpu --steps ${STEPS:-5} --warmup ${WARMUP:-1}"
if [ "${LIST:-0}" = 1 ]; then
  timeout -s KILL 60 rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1 || true
fi
run() {  # name, counters...
  local name=$1; shift
  echo "[$(date +%T)] pmc $LINE $name: $*"
  timeout -s KILL 180 rocprofv3 --pmc "$@" -d gpurun_out/pmc_${TAG}_${LINE}_$name -o pmc --output-format csv -- \
    python3 bench.py $ARGS > gpurun_out/pmc_${TAG}_${LINE}_$name.log 2>&1
}
run sq SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE || exit $?
run sq2 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM || exit $?
run fetch FETCH_SIZE || exit $?
run write WRITE_SIZE || exit $?
echo "[$(date +%T)] done"
