// ldsdma_probe: does a wave's in-flight LDS-DMA (global_load_lds_dwordx4) disturb that wave's own
// ds_write / ds_read traffic to OTHER LDS addresses on gfx950?  (DESIGN.md, mlp2v race screen.)
// Each wave, per iteration: issue one 1 KiB LDS-DMA into its region A (HBM-missing source rows),
// then, with the DMA in flight (MODE 0) or after s_waitcnt vmcnt(0) (MODE 1), run K read-modify-
// writes of its region B (disjoint from A); then wait, and check both regions.  Counts mismatches.
// Build: hipcc --offload-arch=gfx950 -O3 -o ldsdma_probe ldsdma_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)p);
}
__device__ __forceinline__ void glds16(const float* gsrc, uint32_t lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}

#define NW 8
#define K 12

template <int MODE>
__global__ void __launch_bounds__(NW * 64) probe(const float* src, int64_t src_floats, int iters, unsigned* bad) {
  __shared__ __attribute__((aligned(16))) float A[NW][256];
  __shared__ __attribute__((aligned(16))) float B[NW][K][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int k = 0; k < K; ++k) B[wave][k][lane] = 0.f;
  __syncthreads();
  unsigned nb = 0, na = 0;
  uint64_t row = ((uint64_t)blockIdx.x * 7919u + wave * 104729u) % (uint64_t)(src_floats / 256);
  for (int it = 0; it < iters; ++it) {
    row = (row * 6364136223846793005ull + 1442695040888963407ull) % (uint64_t)(src_floats / 256);
    const float* g = src + row * 256;
    glds16(g + 4 * lane, lds_addr(&A[wave][0]));
    if (MODE == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < K; ++k) {
      float v = B[wave][k][lane];
      v += 1.f;
      B[wave][k][lane] = v;
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    // region A must hold the source row, region B exactly it + 1 in every slot
    const float4 a = *(const float4*)&A[wave][4 * lane];
    const float4 e = *(const float4*)(g + 4 * lane);
    na += (a.x != e.x) | (a.y != e.y) | (a.z != e.z) | (a.w != e.w);
#pragma unroll
    for (int k = 0; k < K; ++k) nb += B[wave][k][lane] != (float)(it + 1);
    // resynchronise B so one lost write is counted once
#pragma unroll
    for (int k = 0; k < K; ++k) B[wave][k][lane] = (float)(it + 1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  if (nb) atomicAdd(&bad[0], nb);
  if (na) atomicAdd(&bad[1], na);
}

int main(int argc, char** argv) {
  const int grid = argc > 1 ? atoi(argv[1]) : 2048;
  const int iters = argc > 2 ? atoi(argv[2]) : 2000;
  const int reps = argc > 3 ? atoi(argv[3]) : 5;
  const int64_t nf = (int64_t)1 << 28;  // 1 GiB source: HBM misses
  float* src;
  unsigned* bad;
  if (hipMalloc(&src, nf * 4) != hipSuccess || hipMalloc(&bad, 8) != hipSuccess) return 2;
  float* h = (float*)malloc(1 << 24);
  for (int i = 0; i < (1 << 22); ++i) h[i] = (float)(i * 2654435761u % 1000003u);
  for (int64_t o = 0; o < nf; o += (1 << 22)) hipMemcpy(src + o, h, 1 << 24, hipMemcpyHostToDevice);
  for (int mode = 0; mode < 2; ++mode) {
    for (int r = 0; r < reps; ++r) {
      hipMemset(bad, 0, 8);
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      hipEventRecord(e0);
      if (mode == 0) hipLaunchKernelGGL(probe<0>, dim3(grid), dim3(NW * 64), 0, 0, src, nf, iters, bad);
      else hipLaunchKernelGGL(probe<1>, dim3(grid), dim3(NW * 64), 0, 0, src, nf, iters, bad);
      hipEventRecord(e1);
      unsigned hb[2];
      if (hipMemcpy(hb, bad, 8, hipMemcpyDeviceToHost) != hipSuccess) return 3;
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      printf("mode %d (%s) rep %d: B mismatches %u, A mismatches %u of %lld writes, %.1f ms\n", mode,
             mode ? "vmcnt(0) before the RMWs" : "RMWs with the LDS-DMA in flight", r, hb[0], hb[1],
             (long long)grid * NW * 64 * K * iters, ms);
      fflush(stdout);
    }
  }
  return 0;
}
