// hpe_fit.hip — one whole training epoch of the reference's 2-layer regressor in ONE launch, for
// the regime the reference actually trains in: 1x1 feature maps (P = 1), batch 128 (Model-96/
// train_96.py:134-140,175-183; Model-88/train_88.py:290-297,355-363; Keras fit over 10^4-10^6 steps).
//
// At P = 1 a step is tiny (128 rows x 96 channels, 36k parameters): launched as train_step + reduce
// + optimizer kernels it is bound by launch and host latency, not by the GPU.  Here the step loop
// runs on the device, and the model is split by HIDDEN UNITS over the workgroups instead of by rows:
//   * workgroup c owns hidden units [32c, 32c+32): its W1 columns (as split-GEMM fragments in every
//     wave's registers and as fp32 master copies + Adam m / v in the owning threads' registers), its
//     b1 entries and W2 rows for the WHOLE epoch — no parameter ever leaves the CU between steps;
//   * forward: Z1 = X.W1[:, c] on MFMA for the batch rows (4 waves x 32-row tiles, X gathered
//     through the epoch permutation by LDS-DMA), A1 = act(Z1 + b1) (+ SpatialDropout), and the
//     workgroup's share of the 3-wide head, A1 . W2[c] per row;
//   * ONE exchange per step: the head partials (rows x 3 floats per workgroup) go to global memory
//     as data-tagged 8-byte granules {value, iteration} (write-through sc1 stores: no fence, no
//     counter); every workgroup polls them and sums all partials in fixed workgroup order
//     (bit-identical predictions in every workgroup);
//   * backward in the same workgroup: MSE gradient, dZ1, dW1 = X^T.dZ1 (MFMA), db1, dW2 — all for
//     the workgroup's own units, so no gradient reduction crosses workgroups; then the Keras legacy
//     optimizer (SGD / Adam / Adamax, L2 on kernels and biases) updates them in registers.
// The GEMMs use the exponent-shifted fp16 split of hpe_common.h (SPLIT) or exact fp32 MFMA; a
// non-finite split accumulator sets a flag and the host re-runs the epoch on the exact path.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/hpe.h"
#include "hpe_common.h"
#include "hpe_dev.h"

#define FIT_NW 4               // waves per workgroup (one per SIMD: 512 VGPRs each)
#define FIT_XS 100             // LDS row stride of an X tile (floats)
#define FIT_XT (32 * FIT_XS)   // floats per X tile
#define FIT_SLOTS 2            // resident X tiles per wave (batch <= 256 stays in LDS across the exchange)
#define FIT_RES_BATCH 256      // batch rows whose X tiles stay resident across the exchange
#define FIT_MAX_BATCH 512      // batch rows: beyond FIT_RES_BATCH the tiles are re-gathered for the
                               // backward and the partial table overlays the X slots
#define FIT_UNION 9216         // floats: A1 park | head-partial table [G][batch][3] | dW1 reduce
#define FIT_POLL 24            // granules in flight per thread in the exchange
#define FIT_PART_OFF 128       // workspace (words): [1] flags, [2..3] debug, [4..4+G) XCC ids, [128..] granules
#define FIT_XCC_OFF 4

enum { FIT_FLAG_NONFINITE = 1, FIT_FLAG_TIMEOUT = 2 };

struct FitArgs {
  const int* prog;
  float* params;
  float* params_t;
  float* m;
  float* v;
  const float* l2;
  const int* tpos;
  const float* x;
  const float* ytrue;
  const int* perm;
  int n, bs, steps, kind;
  float b1, b2, eps;
  const float* alpha;       // [steps] optimizer step sizes (host-computed, as hpe_optim_step)
  uint64_t seed_base;       // dropout seed of step s = seed_base + iter0 + 1 + s
  int64_t iter0;
  float* stats;             // [steps][stats_stride]: sse, sae, reg_0 .. reg_{G-1}
  int stats_stride;
  int* sync;                // workspace
  int spin_limit;           // exchange polls before the timeout flag (< 0: flag at once, tests only)
  int64_t n_params, n_mirror, n_train, n_ws_granules;  // sizes (FIT_DEBUG bounds checks)
  uint64_t* part;           // workspace + FIT_PART_OFF: [2][G][3][bs] granules {float bits, tag}
};

// Barriers after the prefetch of the next step's X tile is issued are LDS-only (bar_lds): a
// __syncthreads() would drain the in-flight LDS-DMA gather (its release fence waits vmcnt(0)).

// LDS layout (floats)
#define FIT_L_XS 0
#define FIT_L_DZ2 (FIT_L_XS + FIT_NW * FIT_SLOTS * FIT_XT)
#define FIT_L_W1T (FIT_L_DZ2 + FIT_MAX_BATCH * 4)       // [96][32] W1 block (post-update)
#define FIT_L_W2T (FIT_L_W1T + 96 * 32)                 // [32][4]  W2 rows
#define FIT_L_B1T (FIT_L_W2T + 128)                     // [32]
#define FIT_L_B2T (FIT_L_B1T + 32)                      // [4]
#define FIT_L_RED (FIT_L_B2T + 4)                       // [4 waves][32][4] dW2 / db1 partials
#define FIT_L_MISC (FIT_L_RED + FIT_NW * 128)           // [48] block reductions + flags
#define FIT_L_UNION (FIT_L_MISC + 48)                   // A1 park [4][16][64] | partials | dW1 reduce [2][3][16][64]
#define FIT_L_END (FIT_L_UNION + FIT_UNION)
#define FIT_LDS_BYTES (FIT_L_END * 4)
static_assert(FIT_LDS_BYTES <= 160 * 1024, "fit kernel LDS");

__device__ __forceinline__ float bsum(float v, float* scratch) {  // block sum, fixed order
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) scratch[threadIdx.x >> 6] = v;
  __syncthreads();
  return (scratch[0] + scratch[1]) + (scratch[2] + scratch[3]);
}

// data-tagged granule: one naturally aligned 8-byte {value, tag} written by ONE sc1 store and read
// by sc1 loads (MI355X_MICROARCH.md, hand-off granules): the tag (the optimizer iteration, >= 1,
// unique per step of an engine) says the value is this step's
// FIT_DEBUG builds check every global index against its buffer and record a violation (code in
// workspace word [2], index in [3]) instead of touching memory out of range
#ifdef FIT_DEBUG
#define FIT_OK(i, bound, code) fit_ok((int64_t)(i), (int64_t)(bound), code, a.sync)
__device__ __forceinline__ bool fit_ok(int64_t i, int64_t bound, int code, int* sync) {
  if (i >= 0 && i < bound) return true;
  __hip_atomic_store(sync + 2, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(sync + 3, (int)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return false;
}
#else
#define FIT_OK(i, bound, code) true
#endif

// same_xcd: every workgroup of the launch sits on one XCD (checked at launch start), whose L2 they
// share: a plain store stays in that L2, where the readers' sc1 loads (which bypass only L1) hit it;
// otherwise write-through sc1 stores (visible to every XCD through memory)
__device__ __forceinline__ void put_granule(uint64_t* p, float v, uint32_t tag, bool same_xcd) {
  const uint64_t g = ((uint64_t)tag << 32) | __float_as_uint(v);
  if (same_xcd)
    __hip_atomic_store(p, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  else
    __hip_atomic_store(p, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t get_granule(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// block sum of 5 values (fixed order), scratch: 32 floats; one LDS-only barrier (the step's
// write-through partial stores need not drain here).  Called once per step: the previous step's
// readers of scratch are three barriers back (pass 2 / reduce / optimizer), so no barrier is
// needed before the writes
__device__ __forceinline__ void bsum5(float (&v)[5], float* scratch) {
#pragma unroll
  for (int k = 0; k < 5; ++k) v[k] = wave_sum_dpp(v[k]);
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int k = 0; k < 5; ++k) scratch[(threadIdx.x >> 6) * 8 + k] = v[k];
  bar_lds();
#pragma unroll
  for (int k = 0; k < 5; ++k) v[k] = (scratch[k] + scratch[8 + k]) + (scratch[16 + k] + scratch[24 + k]);
}

// the Keras legacy optimizer update of one parameter (optim_kernel, hpe_rowprog.hip)
__device__ __forceinline__ void opt_update(int kind, float alpha, float lr, float b1, float b2, float eps,
                                           float g, float& w, float& m, float& v) {
  if (kind == HPE_OPT_SGD) {
    w = w - lr * g;
  } else if (kind == HPE_OPT_ADAM) {
    m += (g - m) * (1.f - b1);
    v += (g * g - v) * (1.f - b2);
    w = w - (m * alpha) / (sqrtf(v) + eps);
  } else {
    m += (g - m) * (1.f - b1);
    v = fmaxf(b2 * v, fabsf(g));
    w = w - alpha * (m / (v + eps));
  }
}

// stage the 32 rows [r0, r0 + 32) of the current batch (clamped to the batch) into an X tile:
// one LDS-DMA dwordx4 per row with Cin/4 lanes active; the source rows come from the epoch
// permutation (lane l looks up row l once)
__device__ __forceinline__ void fit_stage_src(const FitArgs& a, float* xt, int src, int Cin, int lane) {
  const int q = Cin >> 2;
#pragma unroll 4
  for (int r = 0; r < 32; ++r) {
    const int64_t s = (int64_t)__builtin_amdgcn_readlane(src, r);
    if (lane < q && FIT_OK(s, a.n, 2)) glds16(a.x + s * Cin + 4 * lane, lds_addr(xt + r * FIT_XS));
  }
}
// source row of tile row (lane & 31) of the tile at batch row r0 (clamped to the batch)
__device__ __forceinline__ int fit_src(const FitArgs& a, const int* bperm, int r0, int nb, int lane) {
  const int lr = min(r0 + (lane & 31), nb - 1);
  return FIT_OK(bperm - a.perm + lr, a.n, 1) ? bperm[lr] : 0;
}
// as fit_stage_src with the 32 source rows in lanes lo .. lo + 31 of src (two tiles per VGPR)
__device__ __forceinline__ void fit_stage_pair(const FitArgs& a, float* xt, int src, int lo, int Cin, int lane) {
  const int q = Cin >> 2;
#pragma unroll 4
  for (int r = 0; r < 32; ++r) {
    const int64_t s = (int64_t)__builtin_amdgcn_readlane(src, lo + r);
    if (lane < q && FIT_OK(s, a.n, 2)) glds16(a.x + s * Cin + 4 * lane, lds_addr(xt + r * FIT_XS));
  }
}
__device__ __forceinline__ void fit_stage(const FitArgs& a, float* xt, const int* bperm, int r0, int nb, int Cin,
                                          int lane) {
  const int src = fit_src(a, bperm, r0, nb, lane);
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the index load, visibly to the compiler
  fit_stage_src(a, xt, src, Cin, lane);
}

template <int KH, int ACT1, bool SPLIT>
__global__ void __launch_bounds__(FIT_NW * 64) fit_kernel(FitArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int* o = a.prog + a.prog[H_OPS_OFF];
  const int Cin = o[O_K], F = o[O_N];
  const int oW = o[O_W], oB = o[O_BIAS], oW2 = o[O_AUX0], oB2 = o[O_AUX1];
  const int act1 = o[O_EACT], drop1 = o[O_EDROP], act2 = o[O_AUX2], drop2 = o[O_TBASE];
  const uint32_t thr1 = (uint32_t)o[O_ETHR], thr2 = (uint32_t)o[O_TCOUNT];
  const float keep1 = __int_as_float(o[O_EKEEP]), keep2 = __int_as_float(o[O_F0]);
  const float inv_keep1 = 1.f / keep1;
  // the grid is 8 G workgroups of which those with blockIdx % 8 == 0 work: under the round-robin
  // dispatch over the 8 XCDs they share one XCD (speed only: verified below, never assumed)
  if (blockIdx.x & 7) return;
  const int G = gridDim.x >> 3, c = blockIdx.x >> 3;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, half = lane >> 5, l32 = lane & 31;
  const int n = c * 32 + l32;  // this lane's hidden unit (forward / backward)
  const bool nok = n < F;
  float* xs = lds + FIT_L_XS + wave * FIT_SLOTS * FIT_XT;
  float* dz2 = lds + FIT_L_DZ2;
  float* w1t = lds + FIT_L_W1T;
  float* w2t = lds + FIT_L_W2T;
  float* b1t = lds + FIT_L_B1T;
  float* b2t = lds + FIT_L_B2T;
  float* red = lds + FIT_L_RED;
  float* misc = lds + FIT_L_MISC;
  float* a1p = lds + FIT_L_UNION + wave * 1024;  // pass 1: this wave's A1 park [16][64]
  float* dwr = lds + FIT_L_UNION;                // after pass 2: dW1 reduce [2][3][16][64]
  // exchange: every workgroup's partials [G][3][bs]; batches beyond FIT_RES_BATCH re-gather X for
  // the backward, so their (larger) table overlays the X slots
  const bool bigbatch = a.bs > FIT_RES_BATCH;
  float* ptab = lds + (bigbatch ? FIT_L_XS : FIT_L_UNION);

  // ---- owned parameters (fp32 master in LDS / registers, optimizer state in registers, for the
  //      whole epoch) ----
  // W1: thread (wave w, lane) owns the dW1 accumulator elements g = 4w .. 4w+3 of blocks kb = 0..2:
  //     k = 32 kb + (g & 3) + 8 (g >> 2) + 4 half, unit n; the master value lives in the W1 table
  //     w1t[k][n - 32c] (which the fragments are built from), Adam m / v in registers
  // small: tid < 32 -> b1[32c + tid]; 32 <= tid < 128 -> W2[32c + (tid-32)/3][(tid-32)%3];
  //        128 <= tid < 131 -> b2[tid - 128]: every workgroup carries b2 (the predictions of all
  //        rows need it) and updates it identically from the same db2; workgroup 0 writes it back
  const bool adam = a.kind != HPE_OPT_SGD;
  float om[12], ov[12];
  const float l2w = a.l2[oW];
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const int kb = i >> 2, g = 4 * wave + (i & 3);
    const int k = 32 * kb + (g & 3) + 8 * (g >> 2) + 4 * half;
    const bool ok = k < Cin && nok;
    const int gi = oW + k * F + n;
    const bool okd = ok && FIT_OK(gi, a.n_train, 3);
    om[i] = okd && adam ? a.m[gi] : 0.f;
    ov[i] = okd && adam ? a.v[gi] : 0.f;
    w1t[k * 32 + l32] = okd ? a.params[gi] : 0.f;
  }
  int sidx = -1, skind = 0, sn = 0, sj = 0;
  if (tid < 32) {
    sn = tid; skind = 1;
    if (c * 32 + sn < F && oB >= 0) sidx = oB + c * 32 + sn;
  } else if (tid < 128) {
    sn = (tid - 32) / 3; sj = (tid - 32) % 3; skind = 2;
    if (c * 32 + sn < F) sidx = oW2 + (c * 32 + sn) * 3 + sj;
  } else if (tid < 131 && oB2 >= 0) {
    sj = tid - 128; skind = 3; sidx = oB2 + sj;
  }
  if (sidx >= 0 && !FIT_OK(sidx, a.n_train, 4)) sidx = -1;
  float sw = sidx >= 0 ? a.params[sidx] : 0.f;
  float sm = sidx >= 0 && adam ? a.m[sidx] : 0.f;
  float sv = sidx >= 0 && adam ? a.v[sidx] : 0.f;
  const float sl2 = sidx >= 0 ? a.l2[sidx] : 0.f;
  if (tid < 128) w2t[tid] = 0.f;
  if (tid < 32) b1t[tid] = 0.f;
  if (tid < 4) b2t[tid] = 0.f;
  if (tid < 48) misc[tid] = 0.f;
  if (tid < 96 && Cin < 96 && tid >= Cin)  // pad rows of the W1 table
    for (int j = 0; j < 32; ++j) w1t[tid * 32 + j] = 0.f;
  // pad channels [Cin, 96) of every X tile: the staging never writes them; batches > 256 overlay
  // the partial table on the X slots, so pass 2 re-zeroes them after each exchange
  for (int r = tid; r < FIT_NW * FIT_SLOTS * 32; r += blockDim.x)
    for (int col = Cin; col < 96; ++col) lds[FIT_L_XS + r * FIT_XS + col] = 0.f;
  __syncthreads();
  if (sidx >= 0) {
    if (skind == 1) b1t[sn] = sw;
    if (skind == 2) w2t[sn * 4 + sj] = sw;
    if (skind == 3) b2t[sj] = sw;
  }
  __syncthreads();

  // one-time placement check: every workgroup publishes its XCC id; same_xcd iff all are equal
  if (tid == 0) {
    const int xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);  // hwreg(HW_REG_XCC_ID, 0, 4)
    __hip_atomic_store(a.sync + FIT_XCC_OFF + c, xcc + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int same = 1;
    for (int cc = 0; cc < G; ++cc) {
      int v, it = 0;
      while ((v = __hip_atomic_load(a.sync + FIT_XCC_OFF + cc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0 &&
             ++it < (1 << 22))
        __builtin_amdgcn_s_sleep(1);
      same &= v == xcc + 1;
    }
    misc[41] = same ? 1.f : 0.f;
  }
  __syncthreads();
  const bool same_xcd = misc[41] != 0.f;
  bool bad = false;
  int flags = 0;
  float alpha = a.alpha[0];  // (steps >= 1)  // the next step's is loaded one step ahead
  const bool onetile = a.bs <= 32 * FIT_NW;  // every step: at most one tile per wave
#ifdef FIT_STAMPS
  uint64_t ph[10] = {};
  uint64_t tprev = __builtin_amdgcn_s_memtime();
#define FSTAMP(i) do { const uint64_t t_ = __builtin_amdgcn_s_memtime(); ph[i] += t_ - tprev; tprev = t_; } while (0)
#else
#define FSTAMP(i) do {} while (0)
#endif
  for (int s = 0; s < a.steps; ++s) {
    const int b0 = s * a.bs;
    const int nb = min(a.bs, a.n - b0);
    const int ntile = (nb + 31) / 32;
    const int* bperm = a.perm + b0;
    const float inv_count = 1.f / (float)(nb * 3);
    const uint64_t seed = a.seed_base + (uint64_t)(a.iter0 + 1 + s);
    const int tw = (ntile - wave + FIT_NW - 1) / FIT_NW;  // tiles of this wave: wave, wave + 4, ...
    const bool resident = !bigbatch && ntile <= FIT_NW * FIT_SLOTS;

    // ---- this step's weight fragments (from the post-update tables) ----
    SplitW wsp[SPLIT ? 6 : 1];
    float wreg[SPLIT ? 1 : KH];
    float inv1 = 1.f, s2 = 1.f;
    const f32x4 w2v = *(const f32x4*)(w2t + l32 * 4);
    const float b1n = b1t[l32];
    if constexpr (SPLIT) {
      f32x8 v[6];
      float mx = 0.f;
#pragma unroll
      for (int q = 0; q < 6; ++q)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = half * KH + 8 * q + j;
          v[q][j] = (8 * q + j < KH && k < 96) ? w1t[k * 32 + l32] : 0.f;
          mx = fmaxf(mx, fabsf(v[q][j]));
        }
      mx = fmaxf(mx, xor32(mx));
      const float s1 = pow2_scale(mx, 13);
      inv1 = SPLIT_INV_C / s1;
#pragma unroll
      for (int q = 0; q < 6; ++q) wsp[q] = split_w8(v[q] * s1);
      s2 = pow2_scale(fmaxf(fmaxf(fabsf(w2v.x), fabsf(w2v.y)), fabsf(w2v.z)), 2);
    } else {
#pragma unroll
      for (int m = 0; m < KH; ++m) wreg[m] = w1t[(half * KH + m) * 32 + l32];
    }

    // Z1 of one 32-row tile for this lane's unit: acc[g] <-> tile row (g & 3) + 8 (g >> 2) + 4 half
    auto forward = [&](const float* xt) {
      f32x16 acc = {};
      const float* ap = xt + l32 * FIT_XS + half * KH;
      if constexpr (SPLIT) {
#pragma unroll
        for (int q = 0; q < 6; ++q) {
          const f32x4 a0 = *(const f32x4*)(ap + 8 * q), a1 = *(const f32x4*)(ap + 8 * q + 4);
          acc = mfma3_dw(split_d8(f32x8{a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w}), wsp[q], acc);
        }
      } else {
#pragma unroll
        for (int m = 0; m < KH; m += 4) {
          const f32x4 av = *(const f32x4*)(ap + m);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, wreg[m + 0], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, wreg[m + 1], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.z, wreg[m + 2], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av.w, wreg[m + 3], acc, 0, 0, 0);
        }
      }
      return acc;
    };
    // A1 (after dropout) of a tile starting at batch row r0; keep bits in *km
    auto activate = [&](f32x16& acc, int r0, uint32_t& km) {
      if (SPLIT) bad |= !(fabsf(sum16(acc)) <= 3.0e38f);
      km = 0;
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int r = r0 + (g & 3) + 8 * (g >> 2) + 4 * half;
        float z = act1_f<ACT1, SPLIT>(act1, SPLIT ? fmaf(acc[g], inv1, b1n) : acc[g] + b1n);
        if (drop1 >= 0) {
          const bool kp = drop_hash(seed, drop1, (uint64_t)r, n) >= thr1;
          km |= kp ? (1u << g) : 0u;
          z = kp ? z * inv_keep1 : 0.f;
        } else {
          km |= 1u << g;
        }
        acc[g] = nok ? z : 0.f;
      }
    };

    const float alpha_next = FIT_OK(min(s + 1, a.steps - 1), a.steps, 5) ? a.alpha[min(s + 1, a.steps - 1)] : 0.f;
    // the next step's tile sources (one tile per wave), loaded before this step's partial stores so
    // the prefetch below never waits for those write-through stores to drain
    const int nb1 = min(a.bs, a.n - b0 - a.bs);
    const bool pf = onetile && s + 1 < a.steps && wave < (nb1 + 31) / 32;
    const int pf_src = pf ? fit_src(a, bperm + a.bs, 32 * wave, nb1, lane) : 0;
    FSTAMP(0);
    // ---- pass 1: forward of this wave's tiles + this workgroup's head partials ----
    // one tile per wave (batch <= 128, the reference's): X tiles alternate slots by step parity and
    // the next step's tile is prefetched during this step's backward; A1 stays in registers
    const uint32_t tag = (uint32_t)(a.iter0 + 1 + s);
    uint64_t* part_out = a.part + ((size_t)(s & 1) * G + c) * a.bs * 3;  // [3][bs]
    // several tiles per wave (batch > 128): the source rows of all of them are looked up at once
    // (two tiles per VGPR: tile i's row r in lane 32 (i & 1) + r of srcp[i >> 1]), and tile i + 1
    // streams in while tile i computes (32 LDS-DMA pieces per tile: vmcnt(32) = tile i landed)
    f32x16 a1keep = {};
    uint32_t kmkeep = 0;
    int srcp0 = 0, srcp1 = 0;
    if (!onetile) {
      const int r32 = lane & 31, hi = lane >> 5;
      if (hi < tw) srcp0 = fit_src(a, bperm, 32 * (wave + FIT_NW * hi), nb, r32);
      if (2 + hi < tw) srcp1 = fit_src(a, bperm, 32 * (wave + FIT_NW * (2 + hi)), nb, r32);
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the index loads
      if (tw > 0) fit_stage_pair(a, xs, srcp0, 0, Cin, lane);
    }
    for (int i = 0; i < tw; ++i) {
      const int t = wave + FIT_NW * i;
      float* xt = xs + (onetile ? (s & 1) : (resident ? i : (i & 1))) * FIT_XT;
      if (onetile) {
        if (s == 0) fit_stage(a, xt, bperm, 32 * t, nb, Cin, lane);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else if (i + 1 < tw) {
        fit_stage_pair(a, xs + (resident ? i + 1 : ((i + 1) & 1)) * FIT_XT, (i + 1) >= 2 ? srcp1 : srcp0,
                       ((i + 1) & 1) * 32, Cin, lane);
        asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      f32x16 acc = forward(xt);
      uint32_t km;
      activate(acc, 32 * t, km);
      if (onetile) {
        a1keep = acc;
        kmkeep = km;
      }
#pragma unroll
      for (int g = 0; g < 16; ++g) a1p[g * 64 + lane] = acc[g];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      // row-on-lane dot of A1[r][16 h .. 16 h + 16) with W2 (row r = l32), halves combined
      const int r = l32, hh = (r >> 2) & 1, gr = (r & 3) + 4 * (r >> 3);
      const float* ar = a1p + gr * 64 + hh * 32 + 16 * half;
      const float* wr = w2t + 16 * half * 4;
      float p0 = 0.f, p1 = 0.f, p2 = 0.f;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const float av = ar[e];
        const f32x4 w = *(const f32x4*)(wr + e * 4);
        p0 = fmaf(av, w.x, p0);
        p1 = fmaf(av, w.y, p1);
        p2 = fmaf(av, w.z, p2);
      }
      p0 += xor32(p0);
      p1 += xor32(p1);
      p2 += xor32(p2);
      const int R = 32 * t + r;
      if (half == 0 && R < nb && FIT_OK((part_out - a.part) + 2 * a.bs + R, a.n_ws_granules, 6)) {
        put_granule(part_out + R, p0, tag, same_xcd);
        put_granule(part_out + a.bs + R, p1, tag, same_xcd);
        put_granule(part_out + 2 * a.bs + R, p2, tag, same_xcd);
      }
      __builtin_amdgcn_wave_barrier();  // a1p reuse by the next tile
    }

    FSTAMP(1);
    // ---- the step's one exchange: all 256 threads poll the G x rows x 3 tagged partials (8 loads
    //      in flight per thread, re-polled in rounds) into an LDS table; then per row: prediction,
    //      loss sums, dL/dpred (unnormalised 2 (p - y)) ----
    float red5[5] = {0.f, 0.f, 0.f, 0.f, 0.f};  // sse, sae, db2[3]
    // this thread's row label (batch <= 256 = threads: at most one row each), loaded now so its two
    // dependent global reads overlap the exchange
    // rows <= 128: two threads per row (lane pairs l, l ^ 32 of wave r / 32), each summing every
    // other workgroup's partials below; the halves meet in fixed order (even c + odd c), so every
    // workgroup gets the same p
    const bool pair = ntile * 32 * 2 <= FIT_NW * 64;
    const int rr = pair ? ((tid >> 6) << 5) + (tid & 31) : tid;
    // (batch > 256: rows rr and rr + 256)
    float ylab[2][3] = {{0.f, 0.f, 0.f}, {0.f, 0.f, 0.f}};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int ry = rr + h * FIT_NW * 64;
      if (ry < nb) {
        const int src = FIT_OK(bperm - a.perm + ry, a.n, 8) ? bperm[ry] : 0;
        if (FIT_OK(src, a.n, 9)) {
          ylab[h][0] = a.ytrue[(int64_t)src * 3 + 0];
          ylab[h][1] = a.ytrue[(int64_t)src * 3 + 1];
          ylab[h][2] = a.ytrue[(int64_t)src * 3 + 2];
        }
      }
    }
    bar_lds();  // every wave's pass 1 done with its A1 park (ptab overlays it)
    {
      // thread (part, row r): granules gi = c * 3 + j = part, part + TPR, ... of row r, all in
      // flight at once (one memory round trip when the partials are there), into ptab[gi][r]
      const uint64_t* part_in = a.part + (size_t)(s & 1) * G * a.bs * 3;
      const int Rp = ntile * 32, TPR = max(1, (FIT_NW * 64) / Rp);
      const int part = tid / Rp, r0 = tid - part * Rp;
      const int ngr = 3 * G;
      // batches beyond 256 rows: one part per thread, rows tid and tid + 256
      for (int r = r0; part < TPR && r < nb; r += FIT_NW * 64) {
        for (int gi0 = part; gi0 < ngr; gi0 += TPR * FIT_POLL) {
          uint64_t gv[FIT_POLL];
          uint32_t pending = 0;
#pragma unroll
          for (int u = 0; u < FIT_POLL; ++u) {
            const int gi = gi0 + u * TPR;
            if (gi < ngr) {
              pending |= 1u << u;
              gv[u] = FIT_OK((size_t)gi * a.bs + r, a.n_ws_granules, 7) ? get_granule(part_in + (size_t)gi * a.bs + r)
                                                                      : ((uint64_t)tag << 32);
            }
          }
          int it = 0;
          while (true) {
#pragma unroll
            for (int u = 0; u < FIT_POLL; ++u) {
              if (((pending >> u) & 1u) && (uint32_t)(gv[u] >> 32) == tag) {
                ptab[(gi0 + u * TPR) * a.bs + r] = __uint_as_float((uint32_t)gv[u]);
                pending &= ~(1u << u);
              }
            }
            if (!pending) break;
#ifdef FIT_STAMPS
            if (tid == 0) ph[7] += 1;
#endif
            if (++it > a.spin_limit) { flags |= FIT_FLAG_TIMEOUT; break; }
            __builtin_amdgcn_s_sleep(1);
#pragma unroll
            for (int u = 0; u < FIT_POLL; ++u)
              if ((pending >> u) & 1u) gv[u] = get_granule(part_in + (size_t)(gi0 + u * TPR) * a.bs + r);
          }
        }
      }
    }
    if (a.spin_limit < 0) flags |= FIT_FLAG_TIMEOUT;
    if (flags & FIT_FLAG_TIMEOUT) misc[40] = 1.f;
    FSTAMP(8);
    bar_lds();
    FSTAMP(9);
    if (misc[40] != 0.f) { flags |= FIT_FLAG_TIMEOUT; break; }
    const int cpar = pair ? half : 0, cstep = pair ? 2 : 1;
    for (int r = rr, h = 0; r < ntile * 32 && (!pair || r < 128); r += blockDim.x, ++h) {
      f32x4 d = {0.f, 0.f, 0.f, 0.f};
      {
        float p[3] = {0.f, 0.f, 0.f};
        for (int cc = cpar; cc < G; cc += cstep) {
          const float* q = ptab + cc * 3 * a.bs + r;
          p[0] += q[0];
          p[1] += q[a.bs];
          p[2] += q[2 * a.bs];
        }
        if (pair) {
          const float o0 = xor32(p[0]), o1 = xor32(p[1]), o2 = xor32(p[2]);
          p[0] = half ? o0 + p[0] : p[0] + o0;
          p[1] = half ? o1 + p[1] : p[1] + o1;
          p[2] = half ? o2 + p[2] : p[2] + o2;
        }
        p[0] += b2t[0];
        p[1] += b2t[1];
        p[2] += b2t[2];
        if (r < nb && (!pair || half == 0)) {
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          float pj = act_f(act2, p[j]);
          bool k2 = true;
          if (drop2 >= 0) {
            k2 = drop_hash(seed, drop2, (uint64_t)r, j) >= thr2;
            pj = k2 ? pj / keep2 : 0.f;
          }
          const float err = pj - ylab[h][j];
          red5[0] = fmaf(err, err, red5[0]);
          red5[1] += fabsf(err);
          float gj = 2.f * err;
          if (drop2 >= 0) gj = k2 ? gj / keep2 : 0.f;
          if (act2 != ACT_LINEAR) gj *= act_grad(act2, drop2 >= 0 && k2 ? pj * keep2 : pj, p[j]);
          d[j] = gj;
          red5[2 + j] += gj;
        }
        }
      }
      if (!pair || half == 0) *(f32x4*)(dz2 + r * 4) = d;
    }
    FSTAMP(2);
    bsum5(red5, misc);  // its barriers also publish the dz2 table
    float db2[3] = {red5[2], red5[3], red5[4]};
    if (c == 0 && tid == 0 && FIT_OK(s, a.steps, 10)) {
      a.stats[(size_t)s * a.stats_stride + 0] = red5[0];
      a.stats[(size_t)s * a.stats_stride + 1] = red5[1];
    }
    // prefetch the next step's tile (one tile per wave): lands during this step's backward
    if (pf) fit_stage_src(a, xs + ((s + 1) & 1) * FIT_XT, pf_src, Cin, lane);

    FSTAMP(3);
    // ---- pass 2: backward of this wave's tiles: dZ1, dW1 (MFMA), dW2, db1 ----
    f32x16 dw[3] = {f32x16{}, f32x16{}, f32x16{}};
    float dw2[3] = {0.f, 0.f, 0.f}, db1 = 0.f;
    // batch > 256: the partial table overlaid the X slots, so the tiles are gathered again
    // (pipelined as in pass 1) and their forward recomputed
    if (bigbatch)  // the table overlaid this wave's 64 X rows (its readers are behind bsum5's barriers)
      for (int col = Cin; col < 96; ++col) xs[lane * FIT_XS + col] = 0.f;
    if (!resident && tw > 0) fit_stage_pair(a, xs, srcp0, 0, Cin, lane);
    for (int i = 0; i < tw; ++i) {
      const int t = wave + FIT_NW * i;
      float* xt = xs + (onetile ? (s & 1) : (resident ? i : (i & 1))) * FIT_XT;
      if (!resident) {
        if (i + 1 < tw) {
          fit_stage_pair(a, xs + ((i + 1) & 1) * FIT_XT, (i + 1) >= 2 ? srcp1 : srcp0, ((i + 1) & 1) * 32, Cin, lane);
          asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      }
      f32x16 acc;
      uint32_t km;
      if (onetile) {
        acc = a1keep;
        km = kmkeep;
      } else {
        acc = forward(xt);
        activate(acc, 32 * t, km);
      }
      float dz[16];
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int r = 32 * t + (g & 3) + 8 * (g >> 2) + 4 * half;
        const f32x4 d = *(const f32x4*)(dz2 + r * 4);
        const float av = acc[g];
        const float da = d.x * w2v.x + d.y * w2v.y + d.z * w2v.z;
        float gz = (km >> g) & 1u ? (drop1 >= 0 ? da * inv_keep1 : da) : 0.f;
        gz = nok ? gz * act1_g<ACT1>(act1, drop1 >= 0 ? av * keep1 : av) : 0.f;
        dw2[0] = fmaf(av, d.x, dw2[0]);
        dw2[1] = fmaf(av, d.y, dw2[1]);
        dw2[2] = fmaf(av, d.z, dw2[2]);
        db1 += gz;
        dz[g] = gz;
      }
      const float* xp = xt + (4 * half) * FIT_XS + l32;
      if constexpr (SPLIT) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          f32x8 dv;
#pragma unroll
          for (int j = 0; j < 8; ++j) dv[j] = dz[8 * q + j] * s2;
          const SplitW dsp = split_w8(dv);
#pragma unroll
          for (int kb = 0; kb < 3; ++kb) {
            f32x8 xv;
#pragma unroll
            for (int j = 0; j < 8; ++j) xv[j] = xp[(16 * q + 8 * (j >> 2) + (j & 3)) * FIT_XS + 32 * kb];
            dw[kb] = mfma3_dw(split_d8(xv), dsp, dw[kb]);
          }
        }
      } else {
#pragma unroll
        for (int kb = 0; kb < 3; ++kb)
#pragma unroll
          for (int g = 0; g < 16; ++g)
            dw[kb] = __builtin_amdgcn_mfma_f32_32x32x2f32(xp[((g & 3) + 8 * (g >> 2)) * FIT_XS + 32 * kb], dz[g],
                                                          dw[kb], 0, 0, 0);
      }
    }
    if (SPLIT) bad |= !(fabsf(sum16(dw[0]) + sum16(dw[1]) + sum16(dw[2])) <= 3.0e38f);

    FSTAMP(4);
    // ---- reduce dW1 over the 4 waves: buffers A = w0 + w2, B = w1 + w3 (fixed order) ----
    {
      float* buf = dwr + (wave & 1) * 3072;
      if (wave < 2) {
#pragma unroll
        for (int kb = 0; kb < 3; ++kb)
#pragma unroll
          for (int g = 0; g < 16; ++g) buf[(kb * 16 + g) * 64 + lane] = dw[kb][g];
      }
      // dW2 / db1: halves combined, then per-wave partials
      float t2[3];
#pragma unroll
      for (int j = 0; j < 3; ++j) t2[j] = dw2[j] + xor32(dw2[j]);
      const float tb = db1 + xor32(db1);
      if (half == 0) *(f32x4*)(red + (wave * 32 + l32) * 4) = f32x4{t2[0], t2[1], t2[2], tb};
      bar_lds();
      if (wave >= 2) {
#pragma unroll
        for (int kb = 0; kb < 3; ++kb)
#pragma unroll
          for (int g = 0; g < 16; ++g) buf[(kb * 16 + g) * 64 + lane] += dw[kb][g];
      }
      bar_lds();
    }

    FSTAMP(5);
    // ---- optimizer on the owned parameters (regularisation loss on the pre-update weights) ----
    const float gsc = SPLIT ? inv_count * (SPLIT_INV_C / s2) : inv_count;
    float reg = 0.f;
    // straight-line over the 12 owned W1 entries (rows k >= Cin / units n >= F hold zeros with
    // zero gradients and zero state, and are not written back: the update keeps them at zero
    // except through L2 of a zero weight, which is zero)
    float wv[12], gv1[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      const int kb = i >> 2, g = 4 * wave + (i & 3);
      const int k = 32 * kb + (g & 3) + 8 * (g >> 2) + 4 * half;
      const int e = (kb * 16 + g) * 64 + lane;
      gv1[i] = dwr[e] + dwr[3072 + e];
      wv[i] = w1t[k * 32 + l32];
    }
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      reg = fmaf(l2w * wv[i], wv[i], reg);
      gv1[i] = fmaf(gv1[i], gsc, 2.f * l2w * wv[i]);
    }
    // one branch on the optimizer kind for the whole block (straight-line updates inside)
    if (a.kind == HPE_OPT_ADAM) {
#pragma unroll
      for (int i = 0; i < 12; ++i) opt_update(HPE_OPT_ADAM, alpha, alpha, a.b1, a.b2, a.eps, gv1[i], wv[i], om[i], ov[i]);
    } else if (a.kind == HPE_OPT_SGD) {
#pragma unroll
      for (int i = 0; i < 12; ++i) opt_update(HPE_OPT_SGD, alpha, alpha, a.b1, a.b2, a.eps, gv1[i], wv[i], om[i], ov[i]);
    } else {
#pragma unroll
      for (int i = 0; i < 12; ++i) opt_update(HPE_OPT_ADAMAX, alpha, alpha, a.b1, a.b2, a.eps, gv1[i], wv[i], om[i], ov[i]);
    }
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      const int kb = i >> 2, g = 4 * wave + (i & 3);
      const int k = 32 * kb + (g & 3) + 8 * (g >> 2) + 4 * half;
      w1t[k * 32 + l32] = wv[i];  // only its owner touches it until the step-end barrier
    }
    if (sidx >= 0) {
      float graw;
      if (skind == 1) {
        const f32x4* rp = (const f32x4*)(red + sn * 4);
        graw = ((rp[0].w + rp[32].w) + (rp[64].w + rp[96].w));
      } else if (skind == 2) {
        const float* rp = red + sn * 4 + sj;
        graw = ((rp[0] + rp[128]) + (rp[256] + rp[384]));
      } else {
        graw = db2[sj];
      }
      if (skind != 3 || c == 0) reg = fmaf(sl2 * sw, sw, reg);
      const float gr = fmaf(graw, inv_count, 2.f * sl2 * sw);
      opt_update(a.kind, alpha, alpha, a.b1, a.b2, a.eps, gr, sw, sm, sv);
    }
    reg = wave_sum_dpp(reg);  // per-wave shares: the host sums stats[s][2:]
    if (lane == 0 && FIT_OK(2 + 4 * c + wave, a.stats_stride, 11)) a.stats[(size_t)s * a.stats_stride + 2 + 4 * c + wave] = reg;
    // post-update tables for the next step's fragments
    if (sidx >= 0) {
      if (skind == 1) b1t[sn] = sw;
      if (skind == 2) w2t[sn * 4 + sj] = sw;
      if (skind == 3) b2t[sj] = sw;
    }
    bar_lds();
    alpha = alpha_next;
    FSTAMP(6);
  }

#ifdef FIT_STAMPS
  if (lane == 0 && (c == 0 || c == G - 1))
    printf("FITSTAMP wg %d wave %d steps %d same_xcd %d: frag %lu pass1 %lu poll %lu pollbar %lu dz2 %lu bsum %lu pass2 %lu reduce %lu opt %lu rounds %lu\n",
           c, wave, a.steps, (int)same_xcd, ph[0], ph[1], ph[8], ph[9], ph[2], ph[3], ph[4], ph[5], ph[6], ph[7]);
#endif
  // ---- epoch end: parameters, transposed mirror and optimizer state back to global memory ----
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const int kb = i >> 2, g = 4 * wave + (i & 3);
    const int k = 32 * kb + (g & 3) + 8 * (g >> 2) + 4 * half;
    if (k >= Cin || !nok) continue;
    const int gi = oW + k * F + n;
    if (!FIT_OK(gi, a.n_train, 12)) continue;
    const float w = w1t[k * 32 + l32];
    a.params[gi] = w;
    const int tp = a.tpos[gi];
    if (tp >= 0 && FIT_OK(tp, a.n_mirror, 13)) a.params_t[tp] = w;
    if (adam) {
      a.m[gi] = om[i];
      a.v[gi] = ov[i];
    }
  }
  if (sidx >= 0 && (skind != 3 || c == 0)) {
    a.params[sidx] = sw;
    const int tp = a.tpos[sidx];
    if (tp >= 0 && FIT_OK(tp, a.n_mirror, 14)) a.params_t[tp] = sw;
    if (adam) {
      a.m[sidx] = sm;
      a.v[sidx] = sv;
    }
  }
  if (bad) flags |= FIT_FLAG_NONFINITE;
  if (flags) __hip_atomic_fetch_or(a.sync + 1, flags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- host side --------------------------------------------------------------------------------
typedef void (*fit_fn)(FitArgs);

template <int KH, bool SPLIT>
static fit_fn fit_pick_act(int act) {
  if (act == ACT_TANH) return fit_kernel<KH, ACT_TANH, SPLIT>;
  if (act == ACT_SOFTSIGN) return fit_kernel<KH, ACT_SOFTSIGN, SPLIT>;
  return fit_kernel<KH, -1, SPLIT>;
}

static fit_fn fit_pick(const int* w, bool split) {
  const int* o = w + w[H_OPS_OFF];
  const int kh = ((o[O_K] + 7) & ~7) / 2;
  if (kh == 44) return split ? fit_pick_act<44, true>(o[O_EACT]) : fit_pick_act<44, false>(o[O_EACT]);
  if (kh == 48) return split ? fit_pick_act<48, true>(o[O_EACT]) : fit_pick_act<48, false>(o[O_EACT]);
  return nullptr;
}

extern "C" int hpe_fit_supported(const hpe_program* p, int32_t batch) {
  if (!p) return 0;
  const int* w = hpe_prog_words(p);
  // residual stacks (hpe_res.hip): one workgroup runs the epoch, any batch
  if (w[H_KIND] == KIND_RES) return w[H_MODE] == MODE_TRAIN && batch >= 1 && res_supported(w) ? 1 : 0;
  if (w[H_KIND] != KIND_MLP2 || w[H_MODE] != MODE_TRAIN) return 0;
  const int* o = w + w[H_OPS_OFF];
  if (o[O_AUX3] != 3 || (o[O_K] & 3) || o[O_K] > 96 || o[O_K] < 4) return 0;
  if (o[O_N] < 1 || (o[O_N] + 31) / 32 > 32) return 0;  // 8 G <= 256 workgroups
  if (!fit_pick(w, true)) return 0;
  const int G = (o[O_N] + 31) / 32;
  if (batch < 1 || batch > FIT_MAX_BATCH) return 0;
  // partial table: the LDS union (resident X) or the X slots (batch > FIT_RES_BATCH)
  if (G * batch * 3 > (batch > FIT_RES_BATCH ? FIT_NW * FIT_SLOTS * FIT_XT : FIT_UNION)) return 0;
  // the G working workgroups spin on each other's partials, so all must be resident at once. The
  // criterion does not depend on the XCD layout: the whole 8 G grid fits the device's resident
  // capacity (occ per CU x CUs), so every workgroup is dispatched without waiting for another to
  // finish. With 8 XCDs (MI355X) the blockIdx % 8 == 0 workers share one XCD; with another XCD
  // count they do not, the launch-start check sees it and the exchange takes the sc1 path.
  int dev = 0, cus = 0, occ = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  fit_fn k = fit_pick(w, true);
  if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, FIT_LDS_BYTES) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)k, FIT_NW * 64, FIT_LDS_BYTES) != hipSuccess)
    return 0;
  return occ >= 1 && 8 * G <= occ * cus;
}

extern "C" size_t hpe_fit_workspace_size(const hpe_program* p, int32_t batch) {
  if (!p) return 0;
  const int* w = hpe_prog_words(p);
  if (w[H_KIND] == KIND_RES) return 64;  // flags only
  const int G = (w[w[H_OPS_OFF] + O_N] + 31) / 32;
  return FIT_PART_OFF * sizeof(int) + (size_t)2 * G * batch * 3 * sizeof(uint64_t);
}

extern "C" int hpe_fit_epoch(const hpe_program* p, float* params, float* params_t, float* m, float* v,
                             const float* l2, const int32_t* tpos, const float* x, const float* y_true,
                             const int32_t* perm, int64_t n, int32_t batch, int32_t kind, float lr, float beta_1,
                             float beta_2, float epsilon, const float* alpha, uint64_t seed_base, int64_t iter0,
                             float* stats, int32_t stats_stride, int32_t exact, void* workspace, void* stream) {
  if (!p || !params || !params_t || !l2 || !tpos || !x || !y_true || !perm || !alpha || !stats || !workspace)
    return hpe_fail(HPE_EINVAL, "hpe_fit_epoch: null argument");
  if (!hpe_fit_supported(p, batch)) return hpe_fail(HPE_EINVAL, "hpe_fit_epoch: program / batch %d not supported", batch);
  if (kind != HPE_OPT_SGD && (!m || !v)) return hpe_fail(HPE_EINVAL, "hpe_fit_epoch: Adam/Adamax need m and v");
  if (kind < HPE_OPT_SGD || kind > HPE_OPT_ADAMAX) return hpe_fail(HPE_EINVAL, "hpe_fit_epoch: unknown optimizer %d", kind);
  if (n < 1 || n > (int64_t)1 << 30) return hpe_fail(HPE_EINVAL, "hpe_fit_epoch: bad row count %lld", (long long)n);
  const int* w = hpe_prog_words(p);
  if (w[H_KIND] == KIND_RES) {
    if (stats_stride < 3) return hpe_fail(HPE_EINVAL, "hpe_fit_epoch: stats_stride %d < 3", stats_stride);
    hipStream_t s = (hipStream_t)stream;
    if (hipMemsetAsync(workspace, 0, hpe_fit_workspace_size(p, batch), s) != hipSuccess)
      return hpe_fail(HPE_ERUNTIME, "hpe_fit_epoch: memset: %s", hipGetErrorString(hipGetLastError()));
    if (res_fit_launch(w, hpe_prog_dwords(p), params, params_t, m, v, l2, tpos, x, y_true, perm, n, batch, kind,
                       beta_1, beta_2, epsilon, alpha, seed_base, iter0, stats, stats_stride, workspace, s))
      return hpe_fail(HPE_ERUNTIME, "hpe_fit_epoch: residual-stack launch failed");
    return HPE_OK;
  }
  const int G = (w[w[H_OPS_OFF] + O_N] + 31) / 32;
  if (stats_stride < 2 + 4 * G) return hpe_fail(HPE_EINVAL, "hpe_fit_epoch: stats_stride %d < %d", stats_stride, 2 + 4 * G);
  FitArgs a = {};
  a.prog = hpe_prog_dwords(p);
  a.params = params; a.params_t = params_t; a.m = m; a.v = v; a.l2 = l2; a.tpos = tpos;
  a.x = x; a.ytrue = y_true; a.perm = perm;
  a.n = (int)n; a.bs = batch; a.steps = (int)((n + batch - 1) / batch); a.kind = kind;
  a.b1 = beta_1;
  a.b2 = beta_2; a.eps = epsilon;
  a.alpha = alpha; a.seed_base = seed_base; a.iter0 = iter0;
  a.stats = stats; a.stats_stride = stats_stride;
  a.n_train = w[H_NPARAMS_TRAIN];
  a.n_params = w[H_NPARAMS];
  a.n_mirror = (int64_t)1 << 40;  // the mirror's size is the compiler's; checked >= 0 only
  a.n_ws_granules = (int64_t)2 * G * batch * 3;
  a.sync = (int*)workspace;
  a.part = (uint64_t*)((float*)workspace + FIT_PART_OFF);
  {
    const char* e = getenv("HPE_FIT_FORCE_TIMEOUT");  // tests: the host's timeout rollback
    a.spin_limit = (e && e[0] == '1') ? -1 : (1 << 22);
  }
  hipStream_t s = (hipStream_t)stream;
  // flags and granules: no tag of an earlier launch (an exact re-run, or iterations restored from
  // a checkpoint) can match this launch's
  if (hipMemsetAsync(workspace, 0, hpe_fit_workspace_size(p, batch), s) != hipSuccess)
    return hpe_fail(HPE_ERUNTIME, "hpe_fit_epoch: memset: %s", hipGetErrorString(hipGetLastError()));
  fit_fn k = fit_pick(w, !exact && !hpe_exact_fp32());
  if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, FIT_LDS_BYTES) != hipSuccess)
    return hpe_fail(HPE_ERUNTIME, "hpe_fit_epoch: LDS attribute: %s", hipGetErrorString(hipGetLastError()));
  hipLaunchKernelGGL(k, dim3(8 * G), dim3(FIT_NW * 64), FIT_LDS_BYTES, s, a);
  if (hipGetLastError() != hipSuccess) return hpe_fail(HPE_ERUNTIME, "hpe_fit_epoch: launch failed");
  return HPE_OK;
}
