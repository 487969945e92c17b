#!/bin/bash
# PMC passes (separate runs, kernel-trace only) over the BlazeFace timing script
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for PMC in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD" "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_INSTS_MFMA" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $PMC --kernel-trace -d gpurun_out/pmc_blaze_$i -o pmc --output-format csv -- python3 scripts/time_blaze.py 256 > gpurun_out/pmc_blaze_$i.log 2>&1 || exit $?
done
echo done
