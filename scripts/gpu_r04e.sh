#!/bin/bash
# round-4: bounded vs unbounded mismatch at sqnu665j P=64 n=4 — repeat screens
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 240 python -u scripts/diag_bounded.py sqnu665j 64 4 40 > gpurun_out/r04e_b64.log 2>&1; rc=$?; tail -30 gpurun_out/r04e_b64.log; [ $rc = 0 ] || exit $rc
HPE_SPLIT_ONLY=1 timeout -k 10 240 python -u scripts/diag_repeat.py 4 60 sqnu665j 8 > gpurun_out/r04e_rep8s.log 2>&1; rc=$?; tail -12 gpurun_out/r04e_rep8s.log; [ $rc = 0 ] || exit $rc
timeout -k 10 240 python -u scripts/diag_repeat.py 2 40 sqnu665j 96 > gpurun_out/r04e_rep96.log 2>&1; rc=$?; tail -12 gpurun_out/r04e_rep96.log; [ $rc = 0 ] || exit $rc
