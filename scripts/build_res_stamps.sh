#!/bin/bash
# varlibs/libhpe_rst.so: the in-tree objects with the residual-stack kernels built with -DRES_STAMPS
# (per-phase s_memtime sums printed by the whole-epoch kernel); GPU runs select it via HPE_LIB.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
CS=$ROOT/head-pose-estimation-model_amd/csrc
make -C $CS -j8 >/dev/null
mkdir -p $ROOT/varlibs $CS/build_var
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result -mllvm -amdgpu-use-amdgpu-trackers=1 -DRES_STAMPS $*"
for p in 88 96; do for f in 0 1; do
  /opt/rocm/bin/hipcc $F -DRES_PART=$p -DRES_FAST=$f -c -o $CS/build_var/res${p}_${f}_st.o $CS/hpe_res.hip &
done; done
/opt/rocm/bin/hipcc $F -c -o $CS/build_var/res0_st.o $CS/hpe_res.hip &
wait
objs=$(ls $CS/build/*.o | grep -v hpe_res)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $ROOT/varlibs/libhpe_rst.so $objs $CS/build_var/res*_st.o
echo built varlibs/libhpe_rst.so
