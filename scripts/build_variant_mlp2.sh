#!/bin/bash
# Variant library with hpe_mlp2.hip (both objects: default and MLP2_BIG) rebuilt under extra flags:
#   scripts/build_variant_mlp2.sh <name> <flags...>  ->  varlibs/libhpe_<name>.so
set -e
NAME=$1; shift
ROOT=/root/repo; CS=$ROOT/head-pose-estimation-model_amd/csrc; T=$(mktemp -d); cp $CS/build/*.o $T/
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result -mllvm -amdgpu-use-amdgpu-trackers=1 $*"
/opt/rocm/bin/hipcc $F -c -o $T/hpe_mlp2.o $CS/hpe_mlp2.hip 2>/dev/null &
/opt/rocm/bin/hipcc $F -mllvm -amdgpu-disable-unclustered-high-rp-reschedule -mllvm -amdgpu-disable-clustered-low-occupancy-reschedule -Xclang -target-feature -Xclang -packed-fp32-ops -DMLP2_BIG -c -o $T/hpe_mlp2_big.o $CS/hpe_mlp2.hip 2>/dev/null &
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/varlibs/libhpe_$NAME.so $T/*.o; rm -rf $T; echo built $NAME
