#!/bin/bash
# Fast variant library for A/B runs: the in-tree objects with ONE translation unit recompiled
# under extra flags (e.g. -DBFS_PIPE=1), linked to varlibs/libhpe_<name>.so.
# Usage: scripts/build_variant_obj.sh <name> <unit.hip> -- <extra hipcc flags>
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/head-pose-estimation-model_amd/csrc
NAME=$1; UNIT=$2; shift 2
[ "$1" = "--" ] && shift
make -C $CS -j8 >/dev/null
T=$(mktemp -d)
cp $CS/build/*.o $T/
OBJ=$T/${UNIT%.hip}.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result -mllvm -amdgpu-use-amdgpu-trackers=1 "$@" -c -o $OBJ $CS/$UNIT 2>$T/err || { tail -20 $T/err; exit 1; }
mkdir -p $ROOT/varlibs
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/varlibs/libhpe_$NAME.so $(ls $T/*.o)
rm -rf $T
echo built varlibs/libhpe_$NAME.so
