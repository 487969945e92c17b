// HBM stream probe for the chain_split_kernel access pattern (configs[1] inference): every wave of a
// persistent grid (one workgroup per CU) streams 32-row x 384-B tiles (12 x 1 KiB LDS-DMA pieces)
// into its LDS slot(s) and waits for them, with no arithmetic.  Variants: waves per CU, tiles in
// flight per wave (LDS slots), cache policy (aux 0 / nt), busy cycles per tile (s_sleep stands in
// for the MFMA work).  Prints GB/s over a 934 MB buffer (256 images x 9216 rows x 96 fp32).
//   hipcc --offload-arch=gfx950 -O3 scripts/stream_probe.hip -o varlibs/stream_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* gbl_ptr_t;

template <int NW, int DEPTH, int AUX, int SLEEP>
__global__ void __launch_bounds__(NW * 64) probe(const float* x, int64_t ntiles, float* sink) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  float* slot0 = lds + wave * DEPTH * 3072;
  const int64_t gw = (int64_t)blockIdx.x * NW + wave, nw = (int64_t)gridDim.x * NW;
  float acc = 0.f;
  int64_t t = gw;
  auto issue = [&](int64_t tile, int d) {
    const float* src = x + tile * 3072 + 4 * lane;
#pragma unroll
    for (int pc = 0; pc < 12; ++pc)
      __builtin_amdgcn_global_load_lds((gbl_ptr_t)(src + pc * 256), (lds_ptr_t)(slot0 + d * 3072 + pc * 256), 16, 0, AUX);
  };
  // prime DEPTH tiles
#pragma unroll
  for (int d = 0; d < DEPTH; ++d)
    if (t + d * nw < ntiles) issue(t + d * nw, d);
  int d = 0;
  for (; t < ntiles; t += nw) {
    // wait for the oldest tile (DEPTH - 1 younger tiles of 12 pieces stay in flight)
    if (DEPTH == 1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (DEPTH == 2) { if (t + nw < ntiles) asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); else asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
    acc += slot0[d * 3072 + lane];
    if (SLEEP) __builtin_amdgcn_s_sleep(SLEEP);
    if (DEPTH > 1 && t + DEPTH * nw < ntiles) issue(t + DEPTH * nw, d);
    if (DEPTH == 1 && t + nw < ntiles) issue(t + nw, 0);
    d = DEPTH > 1 ? (d + 1) % DEPTH : 0;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (acc == 12345.f) sink[threadIdx.x] = acc;
}

template <int NW, int DEPTH, int AUX, int SLEEP>
void run(const char* name, const float* x, int64_t ntiles, float* sink, int ncu) {
  const int lds = NW * DEPTH * 3072 * 4;
  hipFuncSetAttribute((const void*)probe<NW, DEPTH, AUX, SLEEP>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float best = 1e9f;
  for (int r = 0; r < 6; ++r) {
    hipEventRecord(e0, 0);
    hipLaunchKernelGGL((probe<NW, DEPTH, AUX, SLEEP>), dim3(ncu), dim3(NW * 64), lds, 0, x, ntiles, sink);
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (r > 0 && ms < best) best = ms;
  }
  printf("%-34s %7.3f ms  %6.2f TB/s\n", name, best, ntiles * 3072.0 * 4 / (best * 1e-3) / 1e12);
}

int main() {
  const int64_t ntiles = 256LL * 9216 / 32;   // 73,728 tiles of 12 KiB = 906 MB
  float *x, *sink;
  hipMalloc(&x, ntiles * 3072 * 4);
  hipMalloc(&sink, 4096);
  hipMemset(x, 0, ntiles * 3072 * 4);
  int ncu = 256;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  run<12, 1, 0, 0>("12 waves x 1 tile, default", x, ntiles, sink, ncu);
  run<12, 1, 2, 0>("12 waves x 1 tile, nt", x, ntiles, sink, ncu);
  run<12, 1, 0, 24>("12 waves x 1 tile, sleep 1.5k", x, ntiles, sink, ncu);
  run<6, 2, 0, 0>("6 waves x 2 tiles, default", x, ntiles, sink, ncu);
  run<6, 2, 2, 0>("6 waves x 2 tiles, nt", x, ntiles, sink, ncu);
  run<6, 2, 0, 24>("6 waves x 2 tiles, sleep 1.5k", x, ntiles, sink, ncu);
  run<8, 1, 0, 0>("8 waves x 1 tile, default", x, ntiles, sink, ncu);
  run<4, 2, 0, 0>("4 waves x 2 tiles, default", x, ntiles, sink, ncu);
  run<13, 1, 0, 0>("13 waves x 1 tile, default", x, ntiles, sink, ncu);
  return 0;
}
