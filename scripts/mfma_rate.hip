// MFMA issue-rate probe (gfx950): cycles per instruction of back-to-back fp16 MFMAs on one SIMD,
// one wave per SIMD, 4 independent accumulators.  Decides whether the CDNA3-form
// v_mfma_f32_32x32x8_f16 (BlazeFace kernels) costs the same cycles as the double-K
// v_mfma_f32_32x32x16_f16.   hipcc --offload-arch=gfx950 -O3 scripts/mfma_rate.hip -o /tmp/mfma_rate
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int KIND>
__global__ void probe(float* out, unsigned long long* cyc, int n) {
  const int l = threadIdx.x & 63;
  h4 a4 = {(_Float16)(l * 0.01f), (_Float16)1.f, (_Float16)0.5f, (_Float16)0.25f};
  h8 a8 = {a4.x, a4.y, a4.z, a4.w, a4.x, a4.y, a4.z, a4.w};
  f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  f32x4 d0 = {}, d1 = {}, d2 = {}, d3 = {};
  __builtin_amdgcn_s_barrier();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) {
    if (KIND == 0) {
      c0 = __builtin_amdgcn_mfma_f32_32x32x8f16(a4, a4, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x8f16(a4, a4, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_32x32x8f16(a4, a4, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_32x32x8f16(a4, a4, c3, 0, 0, 0);
    } else if (KIND == 1) {
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, a8, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, a8, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, a8, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, a8, c3, 0, 0, 0);
    } else if (KIND == 2) {
      d0 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, a4, d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, a4, d1, 0, 0, 0);
      d2 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, a4, d2, 0, 0, 0);
      d3 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, a4, d3, 0, 0, 0);
    } else {
      d0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, a8, d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, a8, d1, 0, 0, 0);
      d2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, a8, d2, 0, 0, 0);
      d3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, a8, d3, 0, 0, 0);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int j = 0; j < 16; ++j) s += c0[j] + c1[j] + c2[j] + c3[j];
  for (int j = 0; j < 4; ++j) s += d0[j] + d1[j] + d2[j] + d3[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (l == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

int main() {
  float* out;
  unsigned long long* cyc;
  hipMalloc(&out, 256 * 256 * 4);
  hipMalloc(&cyc, 256 * 4 * 8);
  const int n = 2000;
  const char* names[4] = {"32x32x8f16", "32x32x16_f16", "16x16x16f16", "16x16x32_f16"};
  for (int k = 0; k < 4; ++k) {
    for (int rep = 0; rep < 2; ++rep) {
      if (k == 0) hipLaunchKernelGGL(probe<0>, dim3(1), dim3(256), 0, 0, out, cyc, n);
      if (k == 1) hipLaunchKernelGGL(probe<1>, dim3(1), dim3(256), 0, 0, out, cyc, n);
      if (k == 2) hipLaunchKernelGGL(probe<2>, dim3(1), dim3(256), 0, 0, out, cyc, n);
      if (k == 3) hipLaunchKernelGGL(probe<3>, dim3(1), dim3(256), 0, 0, out, cyc, n);
      hipDeviceSynchronize();
    }
    unsigned long long h[4];
    hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
    printf("%-14s cycles/instr (4 waves, one per SIMD): %.2f %.2f %.2f %.2f\n", names[k], h[0] / (4.0 * n),
           h[1] / (4.0 * n), h[2] / (4.0 * n), h[3] / (4.0 * n));
  }
  return 0;
}
