#!/bin/bash
# Build varlibs/libhpe_<name>.so with both mlp2 objects (default and MLP2_BIG) compiled from
# <mlp2 source> with extra flags (e.g. -DMLP2_STAMPS); GPU A/B runs select it via HPE_LIB.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/head-pose-estimation-model_amd/csrc
NAME=$1; shift; SRC=${1:-$CS/hpe_mlp2.hip}; [ $# -gt 0 ] && shift
mkdir -p $ROOT/varlibs $CS/build_var
make -C $CS -j8 >/dev/null
cp "$SRC" $CS/.var_$NAME.hip
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result -mllvm -amdgpu-use-amdgpu-trackers=1"
SCHED="-mllvm -amdgpu-disable-unclustered-high-rp-reschedule -mllvm -amdgpu-disable-clustered-low-occupancy-reschedule"
/opt/rocm/bin/hipcc $F "$@" -c -o $CS/build_var/mlp2_$NAME.o $CS/.var_$NAME.hip &
/opt/rocm/bin/hipcc $F $SCHED -DMLP2_BIG "$@" -c -o $CS/build_var/mlp2big_$NAME.o $CS/.var_$NAME.hip &
wait
rm -f $CS/.var_$NAME.hip
objs=$(ls $CS/build/*.o | grep -v "hpe_mlp2.o\|hpe_mlp2_big.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/varlibs/libhpe_$NAME.so $objs $CS/build_var/mlp2_$NAME.o $CS/build_var/mlp2big_$NAME.o
echo built varlibs/libhpe_$NAME.so
