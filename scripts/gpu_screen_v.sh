set -o pipefail
echo "== v"; timeout -k 10 300 python -u scripts/diag_repeat.py 2 300 2>&1 | grep -v amdgpu.ids | tail -4 || exit 1
echo "== 12-wave"; HPE_MLP2_V=0 timeout -k 10 300 python -u scripts/diag_repeat.py 2 200 2>&1 | grep -v amdgpu.ids | tail -4 || exit 1
HPE_MLP2_V=0 timeout -k 10 300 python -u scripts/diag_repeat.py 24 30 2>&1 | grep -v amdgpu.ids | tail -4 || exit 1
