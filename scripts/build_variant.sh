#!/bin/bash
# Build varlibs/libhpe_<name>.so: every object from csrc/build except hpe_mlp2.o, which is compiled
# from <mlp2 source> (default: csrc/hpe_mlp2.hip) with extra flags; for GPU A/B runs via HPE_LIB.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/head-pose-estimation-model_amd/csrc
NAME=$1; shift; SRC=${1:-$CS/hpe_mlp2.hip}; [ $# -gt 0 ] && shift
[ -n "$SRC" ] || SRC=$CS/hpe_mlp2.hip
mkdir -p $ROOT/varlibs $CS/build_var
make -C $CS -j8 >/dev/null
cp "$SRC" $CS/.var_$NAME.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result -mllvm -amdgpu-use-amdgpu-trackers=1 "$@" \
  -c -o $CS/build_var/mlp2_$NAME.o $CS/.var_$NAME.hip
rm -f $CS/.var_$NAME.hip
objs=$(ls $CS/build/*.o | grep -v hpe_mlp2.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/varlibs/libhpe_$NAME.so $objs $CS/build_var/mlp2_$NAME.o
echo built varlibs/libhpe_$NAME.so
