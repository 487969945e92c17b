// hpe_dev.h — device helpers shared by the fused regressor kernels (hpe_mlp2.hip, hpe_fit.hip):
// LDS-DMA staging, an LDS-only workgroup barrier, and the layer-1 activations of the hot loops.
#pragma once
#include "hpe_common.h"

// LDS-DMA (global_load_lds) in inline asm: hipcc's waitcnt pass cannot tell the two X buffers
// apart and would put vmcnt(0) before every ds_read of the tile in use, draining the prefetch of
// the next one; hidden from it, the prefetch completes only at the explicit vmcnt(0) before the
// barrier that opens its tile.  M0 is written in the same statement (compiler-reserved).
// the low 32 bits of a flat (generic) pointer into LDS are the LDS byte address (the high half is
// the shared aperture); no generic -> local addrspacecast (its null check miscompiles on constants)
__device__ __forceinline__ uint32_t lds_addr(const float* p) {
  return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)p);
}
// HPE_GLDS_NT: the X stream's pieces non-temporal (read once per launch)
#ifdef HPE_GLDS_NT
#define HPE_GLDS16_OP "global_load_lds_dwordx4 %1, off nt"
#else
#define HPE_GLDS16_OP "global_load_lds_dwordx4 %1, off"
#endif
__device__ __forceinline__ void glds16(const float* gsrc, uint32_t lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t" HPE_GLDS16_OP "\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}
__device__ __forceinline__ void glds4(const float* gsrc, uint32_t lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}

// raw workgroup barrier that waits for LDS traffic only: an in-flight global_load_lds prefetch of
// the next tile survives it (__syncthreads() would drain it with vmcnt(0))
__device__ __forceinline__ void bar_lds() {
  asm volatile("" ::: "memory");       // no LDS access moves across it
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// activation of layer 1 fixed at compile time (tanh: Model-96, softsign: Model-88); ACT1 = -1 is
// the runtime-dispatched variant for the other activations the checkpoints use
// tanh in 5 VALU ops for the fp16-split hot loops, 1 - 2 / (1 + e^{2z}) (e^{2z} -> inf gives 1,
// -> 0 gives -1).  Its error is ABSOLUTE: |fast_tanh5(z) - tanh(z)| <= 2^-22 (2.4e-7) over all z
// (tests/test_gpu_activations.py measures it against float64 through hpe_act_probe), so for
// |z| << 1 the relative error grows (~1e-3 at |z| = 1e-4) where tanhf is relatively accurate.
// The exact-fp32 kernels (the split kernels' overflow twins, HPE_EXACT_FP32=1, the residual-stack
// kernels) use tanhf (FAST = false), so the split-vs-exact error bars are anchored to fp32 tanh.
// Derivative 1 - a^2 as in Keras' TanhGrad.
__device__ __forceinline__ float fast_tanh5(float z) {
  const float e = __builtin_amdgcn_exp2f(z * 2.8853900817779268f);  // 2 log2(e)
  return fmaf(-2.f, __builtin_amdgcn_rcpf(1.f + e), 1.f);
}
template <int ACT1, bool FAST = true>
__device__ __forceinline__ float act1_f(int act, float z) {
  if (ACT1 == ACT_TANH) return FAST ? fast_tanh5(z) : tanhf(z);
  if (ACT1 == ACT_SOFTSIGN) return z * __builtin_amdgcn_rcpf(1.f + fabsf(z));
  return act_f(ACT1 >= 0 ? ACT1 : act, z);
}
template <int ACT1>
__device__ __forceinline__ float act1_g(int act, float a) {
  const int k = ACT1 >= 0 ? ACT1 : act;
  return k == ACT_LINEAR ? 1.f : act_grad(k, a, 0.f);
}

