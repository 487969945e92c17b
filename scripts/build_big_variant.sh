#!/bin/bash
# varlibs/libhpe_<name>.so: the in-tree objects with hpe_mlp2_big.o (the MLP2_BIG object that holds
# mlp2v_kernel) rebuilt with extra flags (e.g. -DMLP2_DIAG_BAR_GME); GPU A/B runs select it via HPE_LIB
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/head-pose-estimation-model_amd/csrc
NAME=$1; shift
make -C $CS -j8 >/dev/null
mkdir -p $ROOT/varlibs $CS/build_var
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result -mllvm -amdgpu-use-amdgpu-trackers=1 \
  -mllvm -amdgpu-disable-unclustered-high-rp-reschedule -mllvm -amdgpu-disable-clustered-low-occupancy-reschedule \
  -DMLP2_BIG "$@" -c -o $CS/build_var/mlp2big_$NAME.o $CS/hpe_mlp2.hip
objs=$(ls $CS/build/*.o | grep -v hpe_mlp2_big.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/varlibs/libhpe_$NAME.so $objs $CS/build_var/mlp2big_$NAME.o
echo built varlibs/libhpe_$NAME.so
