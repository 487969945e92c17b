#!/bin/bash
# Race screen (scripts/diag_repeat.py) of libhpe variants: VARS (varlibs/libhpe_<v>.so, "base" = in-tree)
# at n = 2 (R2 launches) and n = 24 (R24 launches) of the 96x96 training step; optional bench A/B (AB=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
for v in ${VARS:-base}; do
  lib=""; [ "$v" != base ] && lib=$PWD/varlibs/libhpe_$v.so
  echo "== $v"
  HPE_LIB=$lib timeout -k 10 300 python -u scripts/diag_repeat.py 2 ${R2:-200} 2>&1 | grep -v amdgpu.ids | tail -3 || exit 1
  HPE_LIB=$lib timeout -k 10 300 python -u scripts/diag_repeat.py 24 ${R24:-40} 2>&1 | grep -v amdgpu.ids | tail -3 || exit 1
done
if [ "${AB:-0}" = 1 ]; then TAG=scr VARS="$(echo ${VARS} | sed 's/base//')" ROUNDS=2 bash scripts/gpu_ab2.sh; fi
