// hpe_rowprog.hip — the head-pose regression hot path on MI355X (gfx950 / CDNA4).
//
// One persistent kernel interprets a compiled row program (hpe_prog.h) over tiles of T rows
// (positions of the NHWC feature maps, channels-last).  Per tile:
//   * the input rows (T x C_in fp32, contiguous in HBM) are loaded once, coalesced, into LDS;
//   * every 1x1-conv / dense layer runs as fp32 MFMA (v_mfma_f32_32x32x2_f32: exact f32, the
//     reference's fp32 numerics) with A = activations from LDS (ds_read_b128 along K, rows on the
//     lanes, conflict-free row stride) and B = weights from L2 (coalesced 128-B rows);
//   * bias + activation + SpatialDropout are fused into the GEMM epilogue, results go back to LDS;
//   * in training, the loss gradient, every backward GEMM and element-wise backward run on the
//     same LDS tile, and the weight gradients accumulate in MFMA accumulators that stay in
//     registers for the whole launch (each wave owns fixed 32x32 dW blocks); thin layers (N <= 8,
//     e.g. the 3-channel yaw/pitch/roll head) run on the VALU.
// HBM traffic is therefore the compulsory input read (+ 12 B/row output in inference) — the
// intermediate activations of the reference's Keras graph never leave the CU.
//
// Reference semantics restated: Conv2D/Dense + activation (train_96.py:72-92), SpatialDropout2D
// (train_96.py:82,94), Add/Average/Multiply/Activation (attention_model.py:38,56,60,148-149),
// LayerNormalization (attention_model.py:57,61), MSE loss + MAE metric (train_96.py:51-52), the
// autodiff of Keras' fit (train_96.py:175).  Optimizers: Keras legacy SGD/Adam/Adamax.
#include <hip/hip_runtime.h>
#include <atomic>
#include <math.h>
#include <stdlib.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <memory>
#include <mutex>
#include <vector>

#include "hpe_prog.h"
#include "../../include/hpe.h"

#include "hpe_common.h"
#include "hpe_dev.h"



// the (row, column) items of a T x C block over NT threads: thread t takes column t % C and rows
// t / C, t / C + NT / C, ... (one division per thread and op instead of one per item)
template <int NT, typename F>
__device__ __forceinline__ void for_rc(int T, int C, F&& f) {
  if (C <= 0) return;
  if (C <= NT) {
    const int rs = NT / C, r0 = (int)threadIdx.x / C, ch = (int)threadIdx.x - r0 * C;
    if (r0 < rs)
      for (int r = r0; r < T; r += rs) f(r, ch);
  } else {
    for (int it = threadIdx.x; it < T * C; it += NT) {
      const int r = it / C;
      f(r, it - r * C);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// OP_DENSE: out[r][n] = epi(sum_k a[r][k] W[k][n] + b[n]) on fp32 MFMA 32x32x2.
// A[i=row][k] from LDS; contraction split across the lane halves: half h handles k in
// [h*Kh, h*Kh + Kh) (Kh = Cp/2, a multiple of 4) so each lane reads 4 consecutive k with one
// ds_read_b128; slot stride = 4*odd floats makes the 16-row lane groups conflict-free.
// B[k][j=n] = W[k][n]: lanes 0-31 / 32-63 read one contiguous 128-B W row each (L2-resident).
// ------------------------------------------------------------------------------------------------
// SPLIT (inference programs): the weights were split by split_weights_kernel into the MFMA B
// fragments of v_mfma_f32_32x32x16_f16 (hi / scaled-lo fp16, per-column power-of-two scale s1;
// O_AUX3 = float offset in Args::wsplit: [ncb][nks][2][64 lanes x 8 halves], then [ncb * 32]
// 1 / (C s1)); A = 8 consecutive k per lane half (two ds_read_b128), split in registers
// (split_d8); 3 MFMAs (96 cycles) per 16 k instead of 8 exact-fp32 MFMAs (512 cycles), and one
// 16-byte weight load per fragment instead of 16 scalar loads.  A non-finite accumulator (data
// outside the split's range) sets *bad -> the exact-fp32 twin re-runs the launch.
template <int NW>
__device__ __forceinline__ void op_dense_split(const Ctx& c, const pword* o, const float* wsplit, bool& bad) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, half = lane >> 5, l32 = lane & 31;
  const int sa = o[O_A], so = o[O_OUT];
  const int a_off = slot_w(c, sa, S_OFF), a_st = slot_w(c, sa, S_STRIDE);
  const int o_off = slot_w(c, so, S_OFF), o_st = slot_w(c, so, S_STRIDE), o_cp = slot_w(c, so, S_CP);
  const int K = o[O_K], N = o[O_N];
  const int boff = o[O_BIAS];
  const Epi e = load_epi(o);
  const int nrb = c.T >> 5, ncb = (N + 31) >> 5, nks = (K + 15) >> 4;
  const float* base = wsplit + o[O_AUX3];
  const float* invs = base + (size_t)ncb * nks * 512;
  for (int task = wave; task < nrb * ncb; task += NW) {
    const int cb = task / nrb, rb = task - cb * nrb;
    const int n = cb * 32 + l32;
    const bool nok = n < N;
    const float* ap = c.lds + a_off + (rb * 32 + l32) * a_st + 8 * half;
    const h8* bp = (const h8*)(base + (size_t)cb * nks * 512) + lane;
    f32x16 acc = {};
    SplitW wn = {bp[0], bp[64]};
    for (int s = 0; s < nks; ++s) {
      const SplitW w = wn;
      if (s + 1 < nks) wn = SplitW{bp[(s + 1) * 128], bp[(s + 1) * 128 + 64]};
      const f32x4 a0 = *(const f32x4*)(ap + 16 * s), a1 = *(const f32x4*)(ap + 16 * s + 4);
      acc = mfma3_dw(split_d8(f32x8{a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w}), w, acc);
    }
    bad |= !(fabsf(sum16(acc)) <= 3.0e38f);
    if (nok) {
      const float inv = invs[n];
      const float bv = boff >= 0 ? c.params[boff + n] : 0.f;
      const int z_off = e.zslot >= 0 ? slot_w(c, e.zslot, S_OFF) : 0;
      const int z_st = e.zslot >= 0 ? slot_w(c, e.zslot, S_STRIDE) : 0;
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int r = rb * 32 + (g & 3) + 8 * (g >> 2) + 4 * half;
        const float z = fmaf(acc[g], inv, bv);
        c.lds[o_off + r * o_st + n] = epi_fwd(c, e, z, r, n);
        if (e.zslot >= 0) c.lds[z_off + r * z_st + n] = z;
      }
    } else if (n < o_cp) {
#pragma unroll
      for (int g = 0; g < 16; ++g) c.lds[o_off + (rb * 32 + (g & 3) + 8 * (g >> 2) + 4 * half) * o_st + n] = 0.f;
    }
  }
}

// split_weights_kernel: one workgroup per (OP_DENSE op, 32-column block) of an inference program
// (table: {op word offset, split float offset, column block}); the per-column scale from the
// column's max |w| (pow2_scale, as mlp2), then the [nks][2][64][8] fragments of the block
__global__ void __launch_bounds__(256) split_weights_kernel(const int* __restrict__ prog, const int* __restrict__ tab,
                                                            const float* __restrict__ params,
                                                            const float* __restrict__ params_t, float* __restrict__ wsplit) {
  __shared__ float scale[32];
  __shared__ float pmax[8][32];
  const int* t = tab + 3 * blockIdx.x;
  const int* o = prog + t[0];
  const int cb = t[2];
  const int K = o[O_K], N = o[O_N];
  const float* W = (o[O_WSEL] ? params_t : params) + o[O_W];
  const int ncb = (N + 31) >> 5, nks = (K + 15) >> 4;
  float* base = wsplit + t[1];
  {
    // column max |w|: 8 k-groups x 32 columns, then a fixed-order combine
    const int c = threadIdx.x & 31, kg = threadIdx.x >> 5, n = cb * 32 + c;
    float mx = 0.f;
    if (n < N)
      for (int k = kg; k < K; k += 8) mx = fmaxf(mx, fabsf(W[(size_t)k * N + n]));
    pmax[kg][c] = mx;
  }
  __syncthreads();
  if (threadIdx.x < 32) {
    float mx = 0.f;
    for (int kg = 0; kg < 8; ++kg) mx = fmaxf(mx, pmax[kg][threadIdx.x]);
    const float s1 = pow2_scale(mx, 13);
    scale[threadIdx.x] = s1;
    if (cb * 32 + (int)threadIdx.x < ncb * 32) base[(size_t)ncb * nks * 512 + cb * 32 + threadIdx.x] = SPLIT_INV_C / s1;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nks * 64; i += blockDim.x) {
    const int s = i >> 6, lane = i & 63, l32 = lane & 31, h = lane >> 5;
    const int n = cb * 32 + l32;
    f32x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 16 * s + 8 * h + j;
      v[j] = (n < N && k < K) ? W[(size_t)k * N + n] * scale[l32] : 0.f;
    }
    const SplitW w = split_w8(v);
    h8* d = (h8*)(base + ((size_t)cb * nks + s) * 512);
    d[lane] = w.h;
    d[64 + lane] = w.cl;
  }
}

template <int NW>
__device__ __forceinline__ void op_dense(const Ctx& c, const pword* o) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, half = lane >> 5, l32 = lane & 31;
  const int sa = o[O_A], so = o[O_OUT];
  const int a_off = slot_w(c, sa, S_OFF), a_cp = slot_w(c, sa, S_CP), a_st = slot_w(c, sa, S_STRIDE);
  const int o_off = slot_w(c, so, S_OFF), o_st = slot_w(c, so, S_STRIDE), o_cp = slot_w(c, so, S_CP);
  const int K = o[O_K], N = o[O_N];
  const float* W = (o[O_WSEL] ? c.params_t : c.params) + o[O_W];
  const int boff = o[O_BIAS];
  const Epi e = load_epi(o);
  const int nrb = c.T >> 5, ncb = (N + 31) >> 5;
  const int Kh = a_cp >> 1;
  const int kbase = half * Kh;
  const int kval = K - kbase;  // valid k count for this half
  for (int task = wave; task < nrb * ncb; task += NW) {
    const int cb = task / nrb, rb = task - cb * nrb;
    const int n = cb * 32 + l32;
    const bool nok = n < N;
    const float* ap = c.lds + a_off + (rb * 32 + l32) * a_st + kbase;
    const float* bp = W + (size_t)kbase * N + (nok ? n : 0);
    f32x16 acc = {};
    int m = 0;
    // B (weights, L2-resident) is loaded one 8-k step ahead: its latency hides under the previous
    // step's 8 MFMAs instead of stalling every step
    float bn[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) bn[j] = (nok && j < kval && 8 <= Kh) ? bp[(size_t)j * N] : 0.f;
    for (; m + 8 <= Kh; m += 8) {
      const f32x4 a0 = *(const f32x4*)(ap + m);
      const f32x4 a1 = *(const f32x4*)(ap + m + 4);
      float b[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) b[j] = bn[j];
      if (m + 16 <= Kh) {
#pragma unroll
        for (int j = 0; j < 8; ++j) bn[j] = (nok && m + 8 + j < kval) ? bp[(size_t)(m + 8 + j) * N] : 0.f;
      }
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.x, b[0], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.y, b[1], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.z, b[2], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.w, b[3], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.x, b[4], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.y, b[5], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.z, b[6], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a1.w, b[7], acc, 0, 0, 0);
    }
    for (; m < Kh; m += 4) {
      const f32x4 a0 = *(const f32x4*)(ap + m);
      float b[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = (nok && m + j < kval) ? bp[(size_t)(m + j) * N] : 0.f;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.x, b[0], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.y, b[1], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.z, b[2], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.w, b[3], acc, 0, 0, 0);
    }
    if (nok) {
      const float bv = boff >= 0 ? c.params[boff + n] : 0.f;
      const int z_off = e.zslot >= 0 ? slot_w(c, e.zslot, S_OFF) : 0;
      const int z_st = e.zslot >= 0 ? slot_w(c, e.zslot, S_STRIDE) : 0;
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int r = rb * 32 + (g & 3) + 8 * (g >> 2) + 4 * half;
        const float z = acc[g] + bv;
        c.lds[o_off + r * o_st + n] = epi_fwd(c, e, z, r, n);
        if (e.zslot >= 0) c.lds[z_off + r * z_st + n] = z;
      }
    } else if (n < o_cp) {  // keep the K-padding columns of the output slot zero (LDS reuse)
#pragma unroll
      for (int g = 0; g < 16; ++g) c.lds[o_off + (rb * 32 + (g & 3) + 8 * (g >> 2) + 4 * half) * o_st + n] = 0.f;
    }
  }
}

// zero the padding columns [C, Cp) of a slot just (re)defined: slots share LDS over the op list,
// and the MFMA A-operand reads of OP_DENSE / OP_DIN cover Cp columns
template <int NW>
__device__ __forceinline__ void zero_pads(const Ctx& c, int slot, int C) {
  constexpr int NT = NW * 64;
  const int cp = slot_w(c, slot, S_CP);
  const int np = cp - C;
  if (np <= 0) return;
  const int off = slot_w(c, slot, S_OFF), st = slot_w(c, slot, S_STRIDE);
  for_rc<NT>(c.T, np, [&](int r, int j) { c.lds[off + r * st + C + j] = 0.f; });
}

// ------------------------------------------------------------------------------------------------
// OP_TDENSE: thin layer (N <= 8, e.g. the 3-channel pose head) on the VALU; K split S ways over
// threads, partials through LDS scratch, summed in fixed order (deterministic).
// ------------------------------------------------------------------------------------------------
template <int NW>
__device__ __forceinline__ void op_tdense(const Ctx& c, const pword* o) {
  constexpr int NT = NW * 64;
  const int sa = o[O_A], so = o[O_OUT];
  const int a_off = slot_w(c, sa, S_OFF), a_st = slot_w(c, sa, S_STRIDE);
  const int o_off = slot_w(c, so, S_OFF), o_st = slot_w(c, so, S_STRIDE);
  const int K = o[O_K], N = o[O_N], S = o[O_AUX3];
  const float* W = (o[O_WSEL] ? c.params_t : c.params) + o[O_W];
  const int boff = o[O_BIAS];
  const Epi e = load_epi(o);
  float* scratch = c.lds + o[O_AUX2];  // per-op transient region (liveness-planned)
  const int TN = c.T * N;
  const int kc = (K + S - 1) / S;
  for (int it = threadIdx.x; it < TN * S; it += NT) {
    const int s = it / TN, rn = it - s * TN;
    const int r = rn / N, n = rn - r * N;
    const int k0 = s * kc, k1 = min(K, k0 + kc);
    const float* ap = c.lds + a_off + r * a_st;
    float acc = 0.f;
#pragma unroll 8
    for (int k = k0; k < k1; ++k) acc = fmaf(ap[k], W[k * N + n], acc);
    scratch[it] = acc;
  }
  __syncthreads();
  const int z_off = e.zslot >= 0 ? slot_w(c, e.zslot, S_OFF) : 0, z_st = e.zslot >= 0 ? slot_w(c, e.zslot, S_STRIDE) : 0;
  for_rc<NT>(c.T, N, [&](int r, int n) {
    const int rn = r * N + n;
    float z = 0.f;
    for (int s = 0; s < S; ++s) z += scratch[s * TN + rn];
    if (boff >= 0) z += c.params[boff + n];
    c.lds[o_off + r * o_st + n] = epi_fwd(c, e, z, r, n);
    if (e.zslot >= 0) c.lds[z_off + r * z_st + n] = z;
  });
  zero_pads<NW>(c, so, N);
}

// ------------------------------------------------------------------------------------------------
// OP_EW: element-wise (Add / Average / Multiply / Activation / BatchNorm-affine / depthwise-1x1
// scale / standalone SpatialDropout) with the fused epilogue.
// ------------------------------------------------------------------------------------------------
template <int NW>
__device__ __forceinline__ void op_ew(const Ctx& c, const pword* o) {
  constexpr int NT = NW * 64;
  const int flags = o[O_FLAGS];
  const int C = slot_w(c, o[O_OUT], S_C);
  const int a_off = slot_w(c, o[O_A], S_OFF), a_st = slot_w(c, o[O_A], S_STRIDE);
  const int b_off = (flags & EW_HAS_B) ? slot_w(c, o[O_B], S_OFF) : 0;
  const int b_st = (flags & EW_HAS_B) ? slot_w(c, o[O_B], S_STRIDE) : 0;
  const int o_off = slot_w(c, o[O_OUT], S_OFF), o_st = slot_w(c, o[O_OUT], S_STRIDE);
  const float f0 = __int_as_float(o[O_F0]), f1 = __int_as_float(o[O_F1]);
  const int soff = o[O_AUX0], toff = o[O_AUX1];
  const Epi e = load_epi(o);
  const int z_off = e.zslot >= 0 ? slot_w(c, e.zslot, S_OFF) : 0, z_st = e.zslot >= 0 ? slot_w(c, e.zslot, S_STRIDE) : 0;
  for_rc<NT>(c.T, C, [&](int r, int ch) {
    const float va = c.lds[a_off + r * a_st + ch];
    float v;
    if (flags & EW_MUL) v = va * c.lds[b_off + r * b_st + ch];
    else v = (flags & EW_HAS_B) ? f0 * va + f1 * c.lds[b_off + r * b_st + ch] : f0 * va;
    if (flags & EW_AFFINE) v = v * c.params[soff + ch] + (toff >= 0 ? c.params[toff + ch] : 0.f);
    c.lds[o_off + r * o_st + ch] = epi_fwd(c, e, v, r, ch);
    if (e.zslot >= 0) c.lds[z_off + r * z_st + ch] = v;
  });
  zero_pads<NW>(c, o[O_OUT], C);
}

// ------------------------------------------------------------------------------------------------
// OP_LN: LayerNormalization over channels (two-pass mean/variance in registers, one wave per row,
// wave64 shuffle reductions).  Training keeps xhat and rstd for OP_LNB.
// ------------------------------------------------------------------------------------------------
template <int NW>
__device__ __forceinline__ void op_ln(const Ctx& c, const pword* o) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int C = slot_w(c, o[O_A], S_C);
  const int a_off = slot_w(c, o[O_A], S_OFF), a_st = slot_w(c, o[O_A], S_STRIDE);
  const int o_off = slot_w(c, o[O_OUT], S_OFF), o_st = slot_w(c, o[O_OUT], S_STRIDE);
  const int goff = o[O_AUX0], boff = o[O_AUX1];
  const int xs = o[O_AUX2], rs = o[O_AUX3];
  const float eps = __int_as_float(o[O_F0]);
  const Epi e = load_epi(o);
  const float invC = 1.f / (float)C;
  // gamma / beta of this lane's channels loaded once per op (not once per row: the LDS stores in
  // between keep the compiler from reusing global loads), DPP wave sums (no LDS round trips)
  const int nj = (C + 63) >> 6;   // <= 8
  float gam[8], bet[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int ch = lane + 64 * j;
    gam[j] = (j < nj && ch < C && goff >= 0) ? c.params[goff + ch] : 1.f;
    bet[j] = (j < nj && ch < C && boff >= 0) ? c.params[boff + ch] : 0.f;
  }
  const int xs_off = xs >= 0 ? slot_w(c, xs, S_OFF) : 0, xs_st = xs >= 0 ? slot_w(c, xs, S_STRIDE) : 0;
  const int rs_off = rs >= 0 ? slot_w(c, rs, S_OFF) : 0, rs_st = rs >= 0 ? slot_w(c, rs, S_STRIDE) : 0;
  for (int r = wave; r < c.T; r += NW) {
    float v[8];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int ch = lane + 64 * j;
      v[j] = (j < nj && ch < C) ? c.lds[a_off + r * a_st + ch] : 0.f;
      s += v[j];
    }
    const float mean = wave_sum_dpp(s) * invC;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int ch = lane + 64 * j;
      const float d = (j < nj && ch < C) ? v[j] - mean : 0.f;
      q += d * d;
    }
    const float var = wave_sum_dpp(q) * invC;
    const float rstd = rsqrtf(var + eps);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int ch = lane + 64 * j;
      if (j < nj && ch < C) {
        const float xh = (v[j] - mean) * rstd;
        const float y = fmaf(xh, gam[j], bet[j]);
        c.lds[o_off + r * o_st + ch] = epi_fwd(c, e, y, r, ch);
        if (xs >= 0) c.lds[xs_off + r * xs_st + ch] = xh;
      }
    }
    if (rs >= 0 && lane == 0) c.lds[rs_off + r * rs_st] = rstd;
  }
  zero_pads<NW>(c, o[O_OUT], C);
  if (xs >= 0) zero_pads<NW>(c, xs, C);
}

// ------------------------------------------------------------------------------------------------
// OP_LOSS: e = pred - y; sum e^2, sum |e| over valid rows; dL/dpred = 2 e / count through the
// producer's epilogue (mse: train_96.py:51; labels (B,1,1,3) broadcast over H,W)
// ------------------------------------------------------------------------------------------------
template <int NW>
__device__ __forceinline__ void op_loss(const Ctx& c, const pword* o, const float* __restrict__ ytrue,
                                        const int* __restrict__ idx, float inv_count, bool train,
                                        float& sse, float& sae) {
  constexpr int NT = NW * 64;
  const int N = o[O_N];
  const int a_off = slot_w(c, o[O_A], S_OFF), a_st = slot_w(c, o[O_A], S_STRIDE);
  const int g_off = slot_w(c, o[O_OUT], S_OFF), g_st = slot_w(c, o[O_OUT], S_STRIDE);
  const Epi e = load_epi(o);
  for (int it = threadIdx.x; it < c.T * N; it += NT) {
    const int r = it / N, n = it - r * N;
    const int64_t R = c.row0 + r;
    const float p = c.lds[a_off + r * a_st + n];
    float g = 0.f;
    if (R < c.nrows) {
      const int64_t img = R / c.P;
      const int64_t src = idx ? (int64_t)idx[img] : img;
      const float err = p - ytrue[src * N + n];
      sse = fmaf(err, err, sse);
      sae += fabsf(err);
      g = 2.f * err * inv_count;
    }
    if (train) {
      const float z = e.zslot >= 0 ? c.lds[slot_w(c, e.zslot, S_OFF) + r * slot_w(c, e.zslot, S_STRIDE) + n] : 0.f;
      c.lds[g_off + r * g_st + n] = epi_bwd(c, e, g, p, z, r, n);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// OP_EPIGRAD: out[r][c] <- out[r][c] * epi'(value) in place
// ------------------------------------------------------------------------------------------------
template <int NW>
__device__ __forceinline__ void op_epigrad(const Ctx& c, const pword* o) {
  constexpr int NT = NW * 64;
  const int C = slot_w(c, o[O_OUT], S_C);
  const int v_off = slot_w(c, o[O_A], S_OFF), v_st = slot_w(c, o[O_A], S_STRIDE);
  const int g_off = slot_w(c, o[O_OUT], S_OFF), g_st = slot_w(c, o[O_OUT], S_STRIDE);
  const Epi e = load_epi(o);
  for (int it = threadIdx.x; it < c.T * C; it += NT) {
    const int r = it / C, ch = it - r * C;
    const float z = e.zslot >= 0 ? c.lds[slot_w(c, e.zslot, S_OFF) + r * slot_w(c, e.zslot, S_STRIDE) + ch] : 0.f;
    float* gp = c.lds + g_off + r * g_st + ch;
    *gp = epi_bwd(c, e, *gp, c.lds[v_off + r * v_st + ch], z, r, ch);
  }
}

// destination write of a backward result (STORE / ACCUM / EPIGRAD through the producer of `val`)
__device__ __forceinline__ void dst_write(const Ctx& c, const pword* o, int mode, const Epi& e,
                                          int d_off, int d_st, int v_off, int v_st, int z_off,
                                          int z_st, int r, int ch, float v) {
  float* p = c.lds + d_off + r * d_st + ch;
  if (mode == DST_STORE) *p = v;
  else if (mode == DST_ACCUM) *p += v;
  else {
    const float z = e.zslot >= 0 ? c.lds[z_off + r * z_st + ch] : 0.f;
    *p = epi_bwd(c, e, v, c.lds[v_off + r * v_st + ch], z, r, ch);
  }
}

// ------------------------------------------------------------------------------------------------
// OP_DIN: out[r][k] (=|+=|epigrad) sum_n a[r][n] W[k][n], reading W^T [N][K] (mirror kept by the
// optimizer) so B rows stay coalesced.  Same MFMA tiling as OP_DENSE.
// ------------------------------------------------------------------------------------------------
template <int NW>
__device__ __forceinline__ void op_din(const Ctx& c, const pword* o) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, half = lane >> 5, l32 = lane & 31;
  const int sa = o[O_A], so = o[O_OUT];
  const int a_off = slot_w(c, sa, S_OFF), a_cp = slot_w(c, sa, S_CP), a_st = slot_w(c, sa, S_STRIDE);
  const int d_off = slot_w(c, so, S_OFF), d_st = slot_w(c, so, S_STRIDE), d_cp = slot_w(c, so, S_CP);
  const int K = o[O_K], N = o[O_N], mode = o[O_MODE];
  const int vs = o[O_AUX0];
  const int v_off = vs >= 0 ? slot_w(c, vs, S_OFF) : 0, v_st = vs >= 0 ? slot_w(c, vs, S_STRIDE) : 0;
  const Epi e = load_epi(o);
  const int z_off = e.zslot >= 0 ? slot_w(c, e.zslot, S_OFF) : 0;
  const int z_st = e.zslot >= 0 ? slot_w(c, e.zslot, S_STRIDE) : 0;
  const float* WT = (o[O_WSEL] ? c.params : c.params_t) + o[O_W];
  const int nrb = c.T >> 5, ncb = (K + 31) >> 5;
  const int Nh = a_cp >> 1;
  const int nbase = half * Nh;
  const int nval = N - nbase;
  for (int task = wave; task < nrb * ncb; task += NW) {
    const int cb = task / nrb, rb = task - cb * nrb;
    const int k = cb * 32 + l32;
    const bool kok = k < K;
    const float* ap = c.lds + a_off + (rb * 32 + l32) * a_st + nbase;
    const float* bp = WT + (size_t)nbase * K + (kok ? k : 0);
    f32x16 acc = {};
    float bn[4];  // W^T loaded one 4-n step ahead (latency under the previous step's MFMAs)
#pragma unroll
    for (int j = 0; j < 4; ++j) bn[j] = (kok && j < nval) ? bp[(size_t)j * K] : 0.f;
    for (int m = 0; m < Nh; m += 4) {
      const f32x4 a0 = *(const f32x4*)(ap + m);
      float b[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = bn[j];
      if (m + 4 < Nh) {
#pragma unroll
        for (int j = 0; j < 4; ++j) bn[j] = (kok && m + 4 + j < nval) ? bp[(size_t)(m + 4 + j) * K] : 0.f;
      }
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.x, b[0], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.y, b[1], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.z, b[2], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a0.w, b[3], acc, 0, 0, 0);
    }
    if (kok) {
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int r = rb * 32 + (g & 3) + 8 * (g >> 2) + 4 * half;
        dst_write(c, o, mode, e, d_off, d_st, v_off, v_st, z_off, z_st, r, k, acc[g]);
      }
    } else if (mode == DST_STORE && k < d_cp) {
#pragma unroll
      for (int g = 0; g < 16; ++g) c.lds[d_off + (rb * 32 + (g & 3) + 8 * (g >> 2) + 4 * half) * d_st + k] = 0.f;
    }
  }
}

// OP_TDIN: thin contraction (N <= 8): out[r][k] (=|+=|epigrad) sum_n a[r][n] W[k][n]
template <int NW>
__device__ __forceinline__ void op_tdin(const Ctx& c, const pword* o) {
  constexpr int NT = NW * 64;
  const int sa = o[O_A], so = o[O_OUT];
  const int a_off = slot_w(c, sa, S_OFF), a_st = slot_w(c, sa, S_STRIDE);
  const int d_off = slot_w(c, so, S_OFF), d_st = slot_w(c, so, S_STRIDE);
  const int K = o[O_K], N = o[O_N], mode = o[O_MODE];
  const int vs = o[O_AUX0];
  const int v_off = vs >= 0 ? slot_w(c, vs, S_OFF) : 0, v_st = vs >= 0 ? slot_w(c, vs, S_STRIDE) : 0;
  const Epi e = load_epi(o);
  const int z_off = e.zslot >= 0 ? slot_w(c, e.zslot, S_OFF) : 0;
  const int z_st = e.zslot >= 0 ? slot_w(c, e.zslot, S_STRIDE) : 0;
  const float* W = (o[O_WSEL] ? c.params_t : c.params) + o[O_W];
  for (int it = threadIdx.x; it < c.T * K; it += NT) {
    const int r = it / K, k = it - r * K;
    const float* ap = c.lds + a_off + r * a_st;
    const float* wp = W + (size_t)k * N;
    float v = 0.f;
    for (int n = 0; n < N; ++n) v = fmaf(ap[n], wp[n], v);
    dst_write(c, o, mode, e, d_off, d_st, v_off, v_st, z_off, z_st, r, k, v);
  }
  if (mode == DST_STORE) zero_pads<NW>(c, so, K);
}

// OP_EWB: backward of OP_EW (its epilogue already applied by OP_EPIGRAD / fused producer)
template <int NW>
__device__ __forceinline__ void op_ewb(const Ctx& c, const pword* o) {
  constexpr int NT = NW * 64;
  const int flags = o[O_FLAGS];
  const int C = slot_w(c, o[O_OUT], S_C);
  const int g_off = slot_w(c, o[O_OUT], S_OFF), g_st = slot_w(c, o[O_OUT], S_STRIDE);
  const int a_off = slot_w(c, o[O_A], S_OFF), a_st = slot_w(c, o[O_A], S_STRIDE);
  const int hb = flags & EW_HAS_B;
  const int b_off = hb ? slot_w(c, o[O_B], S_OFF) : 0, b_st = hb ? slot_w(c, o[O_B], S_STRIDE) : 0;
  const int d0 = o[O_AUX0], d1 = o[O_AUX1];
  const int d0_off = d0 >= 0 ? slot_w(c, d0, S_OFF) : 0, d0_st = d0 >= 0 ? slot_w(c, d0, S_STRIDE) : 0;
  const int d1_off = d1 >= 0 ? slot_w(c, d1, S_OFF) : 0, d1_st = d1 >= 0 ? slot_w(c, d1, S_STRIDE) : 0;
  const int mode = o[O_MODE];  // bit0: d0 accumulate, bit1: d1 accumulate
  const float f0 = __int_as_float(o[O_F0]), f1 = __int_as_float(o[O_F1]);
  const int soff = o[O_AUX2];
  for (int it = threadIdx.x; it < c.T * C; it += NT) {
    const int r = it / C, ch = it - r * C;
    float g = c.lds[g_off + r * g_st + ch];
    if (flags & EW_AFFINE) g *= c.params[soff + ch];
    float g0, g1 = 0.f;
    if (flags & EW_MUL) {
      g0 = g * c.lds[b_off + r * b_st + ch];
      g1 = g * c.lds[a_off + r * a_st + ch];
    } else {
      g0 = f0 * g;
      g1 = f1 * g;
    }
    if (d0 >= 0) {
      float* p = c.lds + d0_off + r * d0_st + ch;
      *p = (mode & 1) ? *p + g0 : g0;
    }
    if (d1 >= 0) {
      float* p = c.lds + d1_off + r * d1_st + ch;
      *p = (mode & 2) ? *p + g1 : g1;
    }
  }
  if (d0 >= 0 && !(mode & 1)) zero_pads<NW>(c, d0, C);
  if (d1 >= 0 && !(mode & 2)) zero_pads<NW>(c, d1, C);
}

// OP_LNB: LayerNorm backward, one wave per row
template <int NW>
__device__ __forceinline__ void op_lnb(const Ctx& c, const pword* o) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int C = slot_w(c, o[O_A], S_C);
  const int x_off = slot_w(c, o[O_A], S_OFF), x_st = slot_w(c, o[O_A], S_STRIDE);
  const int g_off = slot_w(c, o[O_B], S_OFF), g_st = slot_w(c, o[O_B], S_STRIDE);
  const int d_off = slot_w(c, o[O_OUT], S_OFF), d_st = slot_w(c, o[O_OUT], S_STRIDE);
  const int goff = o[O_AUX0], rs = o[O_AUX1], mode = o[O_MODE];
  const int rs_off = slot_w(c, rs, S_OFF), rs_st = slot_w(c, rs, S_STRIDE);
  const float invC = 1.f / (float)C;
  for (int r = wave; r < c.T; r += NW) {
    float xh[8], dxh[8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int ch = lane + 64 * j;
      xh[j] = 0.f;
      dxh[j] = 0.f;
      if (ch < C) {
        xh[j] = c.lds[x_off + r * x_st + ch];
        dxh[j] = c.lds[g_off + r * g_st + ch] * (goff >= 0 ? c.params[goff + ch] : 1.f);
      }
      s1 += dxh[j];
      s2 += dxh[j] * xh[j];
    }
    const float m1 = wave_sum(s1) * invC, m2 = wave_sum(s2) * invC;
    const float rstd = c.lds[rs_off + r * rs_st];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int ch = lane + 64 * j;
      if (ch < C) {
        const float v = rstd * (dxh[j] - m1 - xh[j] * m2);
        float* p = c.lds + d_off + r * d_st + ch;
        *p = mode == DST_ACCUM ? *p + v : v;
      }
    }
  }
  if (mode != DST_ACCUM) zero_pads<NW>(c, o[O_OUT], C);
}

// ------------------------------------------------------------------------------------------------
// the kernel
// ------------------------------------------------------------------------------------------------


// GS (global slots): programs whose slot plan exceeds 160 KiB of LDS (the widest residual stacks of
// the reference, e.g. s25l3n04's 512-256-256-... Conv2D stack, H_GSLOTS) keep their tile slots in a
// per-workgroup region of a device scratch buffer instead; the interpreter is unchanged (all slot
// accesses go through c.lds; workgroup-scope barriers order them: one CU, one L1).  Programs with
// more dW blocks than NW * MAXACC accumulators run H_NPASS launches, pass p owning blocks
// [p NW MAXACC, (p+1) NW MAXACC) (the forward / backward is recomputed per pass; every other slab
// entry is written with identical values by each pass).
template <int NW, int MAXACC, bool GS, bool SPLIT = false>
__global__ void __launch_bounds__(NW * 64) rowprog_kernel(Args args) {
  // exact twin of a split launch: runs only when the split kernel flagged a non-finite value
  if (!SPLIT && args.guard && __hip_atomic_load(args.guard, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != args.epoch) return;
  extern __shared__ __attribute__((aligned(16))) float lds_[];
  constexpr int NT = NW * 64;
  const pword* prog = (const pword*)args.prog;
  const int T = prog[H_T];
  const int mode = prog[H_MODE];
  const bool train = mode == MODE_TRAIN;
  const int nops = prog[H_NOPS];
  const int ops_off = prog[H_OPS_OFF];
  const int lds_floats = prog[H_LDS_FLOATS];
  const int in_slot = prog[H_IN_SLOT], out_slot = prog[H_OUT_SLOT];
  const int Cin = prog[H_CIN], Cout = prog[H_COUT];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, half = lane >> 5, l32 = lane & 31;
  float* lds = GS ? args.gscr + (size_t)blockIdx.x * lds_floats : lds_;

  Ctx c;
  c.prog = prog;
  c.params = args.params;
  c.params_t = args.params_t;
  c.lds = lds;
  c.T = T;
  c.nrows = args.nrows;
  c.P = args.P;
  c.img_off = args.img_off;
  c.seed = args.seed;

  for (int i = threadIdx.x; i < lds_floats; i += NT) lds[i] = 0.f;

  f32x16 dacc[MAXACC];
#pragma unroll
  for (int s = 0; s < MAXACC; ++s) dacc[s] = f32x16{};
  float tacc[MAXTHIN];
#pragma unroll
  for (int s = 0; s < MAXTHIN; ++s) tacc[s] = 0.f;
  float sse = 0.f, sae = 0.f;
  bool bad = false;

  const int in_off = slot_w(c, in_slot, S_OFF), in_st = slot_w(c, in_slot, S_STRIDE);
  const int64_t ntiles = (args.nrows + T - 1) / T;
  const bool small = args.nrows < ((int64_t)1 << 31);
  const pword* blk = prog + prog[H_BLK_OFF] + (args.pass * NW + wave) * MAXACC;

  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    c.row0 = tile * T;
    __syncthreads();
    // ---- stage the tile's input rows (coalesced 16-B loads, rows contiguous in HBM) ----
    if ((Cin & 3) == 0) {
      const int q = Cin >> 2, qp = slot_w(c, in_slot, S_CP) >> 2;  // pad columns written as 0
      for_rc<NT>(T, qp, [&](int r, int j) {
        const int64_t R = c.row0 + r;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (R < args.nrows && j < q) {
          int64_t src = R;
          if (args.idx || args.P > 1) {  // 32-bit division when the batch has < 2^31 rows
            const int64_t img = small ? (int64_t)((int)R / args.P) : R / args.P, pos = R - img * args.P;
            src = (args.idx ? (int64_t)args.idx[img] : img) * args.P + pos;
          }
          v = *(const f32x4*)(args.x + src * Cin + 4 * j);
        }
        *(f32x4*)(lds + in_off + r * in_st + 4 * j) = v;
      });
    } else {
      const int cp = slot_w(c, in_slot, S_CP);
      for (int it = threadIdx.x; it < T * cp; it += NT) {
        const int r = it / cp, j = it - r * cp;
        const int64_t R = c.row0 + r;
        float v = 0.f;
        if (R < args.nrows && j < Cin) {
          const int64_t img = R / args.P, pos = R - img * args.P;
          const int64_t src = (args.idx ? (int64_t)args.idx[img] : img) * args.P + pos;
          v = args.x[src * Cin + j];
        }
        lds[in_off + r * in_st + j] = v;
      }
    }
    __syncthreads();
    for (int oi = 0; oi < nops; ++oi) {
      const pword* o = prog + ops_off + oi * O_WORDS;
      const int type = o[O_TYPE];
      switch (type) {
        case OP_DENSE:
          if (SPLIT && o[O_AUX3] >= 0) op_dense_split<NW>(c, o, args.wsplit, bad);
          else op_dense<NW>(c, o);
          break;
        case OP_TDENSE: op_tdense<NW>(c, o); break;
        case OP_EW: op_ew<NW>(c, o); break;
        case OP_LN: op_ln<NW>(c, o); break;
        case OP_LOSS:
          op_loss<NW>(c, o, args.ytrue, args.idx, args.inv_count, train, sse, sae);
          break;
        case OP_EPIGRAD: op_epigrad<NW>(c, o); break;
        case OP_DW: {
          const int sa = o[O_A], sb = o[O_B];
          const int a_off = slot_w(c, sa, S_OFF), a_st = slot_w(c, sa, S_STRIDE);
          const int b_off = slot_w(c, sb, S_OFF), b_st = slot_w(c, sb, S_STRIDE);
          const int K = o[O_K], N = o[O_N];
          const int Th = T >> 1;
#pragma unroll
          for (int s = 0; s < MAXACC; ++s) {
            const int ent = blk[s];
            if (ent >= 0 && (ent >> 16) == oi) {
              const int kb = (ent >> 8) & 0xff, nb = ent & 0xff;
              const int k = kb * 32 + l32, n = nb * 32 + l32;
              const bool kok = k < K, nok = n < N;
              const float* ap = lds + a_off + (half * Th) * a_st + (kok ? k : 0);
              const float* bp = lds + b_off + (half * Th) * b_st + (nok ? n : 0);
              f32x16 acc = dacc[s];
              for (int m = 0; m < Th; m += 4) {
                float a[4], b[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                  a[j] = kok ? ap[(m + j) * a_st] : 0.f;
                  b[j] = nok ? bp[(m + j) * b_st] : 0.f;
                }
#pragma unroll
                for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[j], b[j], acc, 0, 0, 0);
              }
              dacc[s] = acc;
            }
          }
          break;
        }
        case OP_TACC: {
          const int sa = o[O_A], sb = o[O_B];
          const int a_off = sa >= 0 ? slot_w(c, sa, S_OFF) : 0, a_st = sa >= 0 ? slot_w(c, sa, S_STRIDE) : 0;
          const int b_off = slot_w(c, sb, S_OFF), b_st = slot_w(c, sb, S_STRIDE);
          const int N = o[O_N], tm = o[O_AUX3], tb = o[O_TBASE], tn = o[O_TCOUNT];
#pragma unroll
          for (int s = 0; s < MAXTHIN; ++s) {
            const int el = threadIdx.x + s * NT - tb;
            if (el >= 0 && el < tn) {
              int ka, nb_;
              if (tm == TACC_GEMM) { ka = el / N; nb_ = el - ka * N; }
              else { ka = el; nb_ = el; }
              const float* ap = lds + a_off + ka;
              const float* bp = lds + b_off + nb_;
              float acc = 0.f;
              if (tm == TACC_BIAS || sa < 0) {
                for (int r = 0; r < T; ++r) acc += bp[r * b_st];
              } else {
                for (int r = 0; r < T; ++r) acc = fmaf(ap[r * a_st], bp[r * b_st], acc);
              }
              tacc[s] += acc;
            }
          }
          break;
        }
        case OP_DIN: op_din<NW>(c, o); break;
        case OP_TDIN: op_tdin<NW>(c, o); break;
        case OP_EWB: op_ewb<NW>(c, o); break;
        case OP_LNB: op_lnb<NW>(c, o); break;
        default: break;
      }
      __syncthreads();
    }
    if (mode == MODE_FWD) {
      const int o_off = slot_w(c, out_slot, S_OFF), o_st = slot_w(c, out_slot, S_STRIDE);
      for_rc<NT>(T, Cout, [&](int r, int n) {
        const int64_t R = c.row0 + r;
        if (R < args.nrows) args.y[R * Cout + n] = lds[o_off + r * o_st + n];
      });
    }
  }

  if (mode == MODE_FWD) {
    if (SPLIT && bad) __hip_atomic_store(args.guard, args.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  // ---- flush this workgroup's partials: slab[blockIdx] = [dW..., sum e^2, sum |e|] ----
  const int slab = prog[H_SLAB];
  const int npt = prog[H_NPARAMS_TRAIN];
  float* ws = args.ws + (size_t)blockIdx.x * slab;
  if (train) {
#pragma unroll
    for (int s = 0; s < MAXACC; ++s) {
      const int ent = blk[s];
      if (ent >= 0) {
        const pword* o = prog + ops_off + (ent >> 16) * O_WORDS;
        const int K = o[O_K], N = o[O_N], woff = o[O_W];
        const int kb = (ent >> 8) & 0xff, nb = ent & 0xff;
        const int n = nb * 32 + l32;
        if (n < N) {
#pragma unroll
          for (int g = 0; g < 16; ++g) {
            const int k = kb * 32 + (g & 3) + 8 * (g >> 2) + 4 * half;
            if (k < K) ws[woff + k * N + n] = dacc[s][g];
          }
        }
      }
    }
    const int ntacc = prog[H_NTACC];
    const pword* tl = prog + prog[H_TACC_OFF];
#pragma unroll
    for (int s = 0; s < MAXTHIN; ++s) {
      const int e = threadIdx.x + s * NT;
      for (int q = 0; q < ntacc; ++q) {
        const pword* o = prog + ops_off + tl[q] * O_WORDS;
        const int el = e - o[O_TBASE];
        if (el >= 0 && el < o[O_TCOUNT]) ws[o[O_W] + el] = tacc[s];
      }
    }
  }
  // block reduction of the loss sums (fixed order)
  float* red = GS ? lds_ : lds + lds_floats;  // 2 x NW floats past the program's LDS
  const float a = wave_sum(sse), b = wave_sum(sae);
  __syncthreads();
  if (lane == 0) { red[wave] = a; red[NW + wave] = b; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float s0 = 0.f, s1 = 0.f;
    for (int w = 0; w < NW; ++w) { s0 += red[w]; s1 += red[NW + w]; }
    ws[npt] = s0;
    ws[npt + 1] = s1;
  }
}

// grad[i] = sum_g ws[g][i]  (fixed order over workgroups)
// per-workgroup gradient slabs -> flat gradient.  A workgroup owns 64 consecutive parameters;
// wave w sums slabs w, w+4, ... with 4 independent accumulators (16 loads in flight per lane),
// then the 4 wave partials are added in fixed order: deterministic, and ~grid/16 dependent
// latencies instead of grid.
__global__ void __launch_bounds__(256) reduce_kernel(const float* __restrict__ ws, float* __restrict__ grad,
                                                     int grid, int slab, int n) {
  __shared__ float part[4][64];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int i = blockIdx.x * 64 + l;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (i < n) {
    const float* p = ws + i;
    int g = w;
    for (; g + 12 < grid; g += 16) {
      s0 += p[(size_t)g * slab];
      s1 += p[(size_t)(g + 4) * slab];
      s2 += p[(size_t)(g + 8) * slab];
      s3 += p[(size_t)(g + 12) * slab];
    }
    for (; g < grid; g += 4) s0 += p[(size_t)g * slab];
  }
  part[w][l] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (w == 0 && i < n) grad[i] = (part[0][l] + part[1][l]) + (part[2][l] + part[3][l]);
}

// one parameter's sum over the workgroup slabs in exactly reduce_kernel's order (wave w's four
// strided accumulators, then the fixed-order combination of the four wave partials): a fused
// reduce + optimizer launch gives the bit-identical gradient
__device__ __forceinline__ float reduce_slabs(const float* __restrict__ p, int grid, int slab) {
  float part[4];
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int g = w;
    for (; g + 12 < grid; g += 16) {
      s0 += p[(size_t)g * slab];
      s1 += p[(size_t)(g + 4) * slab];
      s2 += p[(size_t)(g + 8) * slab];
      s3 += p[(size_t)(g + 12) * slab];
    }
    for (; g < grid; g += 4) s0 += p[(size_t)g * slab];
    part[w] = (s0 + s1) + (s2 + s3);
  }
  return (part[0] + part[1]) + (part[2] + part[3]);
}

// Keras legacy optimizer update of parameter i from its gradient g (before gscale / L2)
__device__ __forceinline__ float optim_update(int kind, float lr, float alpha, float b1, float b2, float eps,
                                              float gscale, float* __restrict__ w, float* __restrict__ m,
                                              float* __restrict__ v, float graw, float c2, int64_t i, float& reg) {
  const float wi = w[i];
  reg = fmaf(c2 * wi, wi, reg);
  const float g = fmaf(graw, gscale, 2.f * c2 * wi);
  float wn;
  if (kind == HPE_OPT_SGD) {
    wn = wi - lr * g;
  } else if (kind == HPE_OPT_ADAM) {
    float mi = m[i], vi = v[i];
    mi += (g - mi) * (1.f - b1);
    vi += (g * g - vi) * (1.f - b2);
    m[i] = mi;
    v[i] = vi;
    wn = wi - (mi * alpha) / (sqrtf(vi) + eps);
  } else {
    float mi = m[i], vi = v[i];
    mi += (g - mi) * (1.f - b1);
    vi = fmaxf(b2 * vi, fabsf(g));
    m[i] = mi;
    v[i] = vi;
    wn = wi - alpha * (mi / (vi + eps));
  }
  w[i] = wn;
  return wn;
}

// Keras legacy optimizers (TF ApplyGradientDescent / ApplyAdam / ApplyAdaMax functors)
__global__ void optim_kernel(int kind, float lr, float alpha, float b1, float b2, float eps,
                             float gscale, float* __restrict__ w, float* __restrict__ wt,
                             float* __restrict__ m, float* __restrict__ v,
                             const float* __restrict__ grad, const float* __restrict__ l2,
                             const int* __restrict__ tpos, int64_t n, float* __restrict__ regp) {
  float reg = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float wn = optim_update(kind, lr, alpha, b1, b2, eps, gscale, w, m, v, grad[i], l2[i], i, reg);
    const int tp = tpos[i];
    if (tp >= 0) wt[tp] = wn;
  }
  reg = wave_sum(reg);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = reg;
  __syncthreads();
  if (threadIdx.x == 0) regp[2 + blockIdx.x] = red[0] + red[1] + red[2] + red[3];
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // the step's loss sums (post all-reduce)
    regp[0] = grad[n];
    regp[1] = grad[n + 1];
  }
}

// reduce_kernel + optim_kernel in one launch (single-rank per-step training: no all-reduce between
// them): each thread sums its parameter over the workgroup slabs in reduce_kernel's order, keeps
// the flat gradient in grad (same contents as hpe_reduce) and applies the optimizer; block 0 also
// reduces the 4 loss / aux words.  Only for small persistent grids (the P = 1 per-step path: a few
// slabs), where the second launch's latency is a sizable part of the step.
__global__ void __launch_bounds__(256) reduce_optim_kernel(
    const float* __restrict__ ws, int grid, int slab, int kind, float lr, float alpha, float b1, float b2,
    float eps, float gscale, float* __restrict__ w, float* __restrict__ wt, float* __restrict__ m,
    float* __restrict__ v, float* __restrict__ grad, const float* __restrict__ l2, const int* __restrict__ tpos,
    int64_t n, float* __restrict__ regp) {
  float reg = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float gi = reduce_slabs(ws + i, grid, slab);
    grad[i] = gi;
    const float wn = optim_update(kind, lr, alpha, b1, b2, eps, gscale, w, m, v, gi, l2[i], i, reg);
    const int tp = tpos[i];
    if (tp >= 0) wt[tp] = wn;
  }
  reg = wave_sum(reg);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = reg;
  if (blockIdx.x == 0 && threadIdx.x < 4) {
    const float t = reduce_slabs(ws + n + threadIdx.x, grid, slab);
    grad[n + threadIdx.x] = t;
    if (threadIdx.x < 2) regp[threadIdx.x] = t;
  }
  __syncthreads();
  if (threadIdx.x == 0) regp[2 + blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// ------------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------------
static thread_local char g_err[512];

int hpe_fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof g_err, fmt, ap);
  va_end(ap);
  return code;
}
#define fail hpe_fail

#define HIPCHK(x)                                                                      \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) return fail(HPE_ERUNTIME, "%s: %s", #x, hipGetErrorString(e_)); \
  } while (0)

struct hpe_program {
  int* dwords;
  int hdr[H_WORDS];
  int* words;  // host copy (fused-kernel geometry)
  int n_cu;
  int grid_cap;
  int64_t n_words;
  mutable int epoch;  // guarded (fp16-split) launches: guard word = dwords[n_words + epoch % HPE_GUARD_RING]
  float* gscr;        // H_GSLOTS programs: grid_cap x H_LDS_FLOATS slot scratch
  float* wsplit;      // inference programs: OP_DENSE weights split for the fp16 MFMA (null: exact only)
  int* split_tab;     // device {op word offset, split offset, column block} per split workgroup
  int n_split_blocks;
  // gscr / wsplit are one buffer per program: a launch on another stream than the last one that
  // used them waits for that launch (scr_done) instead of sharing the scratch with it
  mutable hipEvent_t scr_done;
  mutable hipStream_t scr_stream;
  mutable bool scr_used;
  mutable std::mutex scr_mu;
};

extern "C" const char* hpe_last_error(void) { return g_err; }

const int* hpe_prog_words(const hpe_program* p) { return p->words; }
const int* hpe_prog_dwords(const hpe_program* p) { return p->dwords; }

static int g_exact = -1;  // -1: not yet read from HPE_EXACT_FP32
bool hpe_exact_fp32() {
  if (g_exact < 0) {
    const char* e = getenv("HPE_EXACT_FP32");
    g_exact = e && e[0] == '1';
  }
  return g_exact == 1;
}

// ---- dominant-kernel timing (hpe_kernel_timing / hpe_kernel_times) ----
// a pool of event pairs recorded around each launch's dominant kernel while timing is on; the
// events are created up front by hpe_kernel_timing, so recording never allocates
static std::vector<hipEvent_t> g_tev;
static int g_tev_cap = 0;
static std::atomic<int> g_tev_n{0};             // slots reserved (hpe_tev_begin)
static std::unique_ptr<std::atomic<uint8_t>[]> g_tev_ok;  // slot's end event recorded (hpe_tev_end)
static int g_tev_ok_cap = 0;
static bool g_tev_on = false;

// reserves the next event pair (launch() may run on several host threads): the slot to pass to
// hpe_tev_end, -1 when timing is off or the pool is full
int hpe_tev_begin(hipStream_t s) {
  if (!g_tev_on) return -1;
  const int slot = g_tev_n.fetch_add(1, std::memory_order_relaxed);
  if (slot >= g_tev_cap) {
    g_tev_n.store(g_tev_cap, std::memory_order_relaxed);
    return -1;
  }
  hipEventRecord(g_tev[2 * slot], s);
  return slot;
}
// called on every path after hpe_tev_begin, failed launches included, so no slot stays half-recorded
void hpe_tev_end(hipStream_t s, int slot) {
  if (slot < 0) return;
  hipEventRecord(g_tev[2 * slot + 1], s);
  g_tev_ok[slot].store(1, std::memory_order_release);
}

extern "C" int hpe_kernel_timing(int32_t capacity) {
  g_tev_on = false;
  g_tev_n = 0;
  if (capacity <= 0) return HPE_OK;
  while ((int)g_tev.size() < 2 * capacity) {
    hipEvent_t e;
    HIPCHK(hipEventCreate(&e));
    g_tev.push_back(e);
  }
  if (g_tev_ok_cap < capacity) {
    g_tev_ok.reset(new std::atomic<uint8_t>[capacity]);
    g_tev_ok_cap = capacity;
  }
  for (int i = 0; i < capacity; ++i) g_tev_ok[i].store(0, std::memory_order_relaxed);
  g_tev_cap = capacity;
  g_tev_on = true;
  return HPE_OK;
}

extern "C" int hpe_kernel_times(float* ms, int32_t max) {
  if (!ms && max > 0) return fail(HPE_EINVAL, "hpe_kernel_times: null argument");
  // the leading run of slots whose end event is recorded (a slot another host thread reserved but
  // has not closed yet ends the run: its end event does not exist yet)
  const int reserved = g_tev_n.load(std::memory_order_relaxed);
  int done = 0;
  while (done < reserved && done < g_tev_cap && g_tev_ok[done].load(std::memory_order_acquire)) ++done;
  const int n = done < max ? done : max;
  for (int i = 0; i < n; ++i) {
    HIPCHK(hipEventSynchronize(g_tev[2 * i + 1]));
    HIPCHK(hipEventElapsedTime(&ms[i], g_tev[2 * i], g_tev[2 * i + 1]));
  }
  return n;
}

// hpe_act_probe: the fused kernels' layer-1 activation (hpe_dev.h act1_f) on a buffer, for the
// error bounds of tests/test_gpu_activations.py
template <int ACT1, bool FAST>
__global__ void act_probe_kernel(int act, const float* z, float* out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = act1_f<ACT1, FAST>(act, z[i]);
}

extern "C" int hpe_act_probe(int32_t act, int32_t fast, const float* z, float* out, int64_t n, void* stream) {
  if (!z || !out || n < 0) return hpe_fail(HPE_EINVAL, "act_probe: bad argument");
  if (act < ACT_LINEAR || act > ACT_LEAKY_RELU) return hpe_fail(HPE_EINVAL, "act_probe: activation %d", act);
  if (n == 0) return HPE_OK;
  const int64_t want = (n + 255) / 256;
  const unsigned grid = (unsigned)(want < 4096 ? want : 4096);
  hipStream_t s = (hipStream_t)stream;
  if (act == ACT_TANH) {
    if (fast) hipLaunchKernelGGL((act_probe_kernel<ACT_TANH, true>), dim3(grid), dim3(256), 0, s, act, z, out, n);
    else hipLaunchKernelGGL((act_probe_kernel<ACT_TANH, false>), dim3(grid), dim3(256), 0, s, act, z, out, n);
  } else if (act == ACT_SOFTSIGN) {
    hipLaunchKernelGGL((act_probe_kernel<ACT_SOFTSIGN, true>), dim3(grid), dim3(256), 0, s, act, z, out, n);
  } else {
    hipLaunchKernelGGL((act_probe_kernel<-1, true>), dim3(grid), dim3(256), 0, s, act, z, out, n);
  }
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? HPE_OK : hpe_fail(HPE_ERUNTIME, "act_probe launch: %s", hipGetErrorString(e));
}

extern "C" int hpe_set_exact_fp32(int on) {
  const int prev = hpe_exact_fp32() ? 1 : 0;
  g_exact = on ? 1 : 0;
  return prev;
}

typedef void (*kfn_t)(Args);

template <int NW, bool GS>
static kfn_t pick_acc(int maxacc) {
  if (maxacc <= 1) return rowprog_kernel<NW, 1, GS>;
  if (maxacc <= 2) return rowprog_kernel<NW, 2, GS>;
  if (maxacc <= 4) return rowprog_kernel<NW, 4, GS>;
  if (maxacc <= 8) return rowprog_kernel<NW, 8, GS>;
  return nullptr;
}

// split instantiation: inference programs (MAXACC 1, LDS slots) on 8 waves
static kfn_t pick_split(int nw, int maxacc) {
  if (maxacc > 1) return nullptr;
  if (nw == 8) return rowprog_kernel<8, 1, false, true>;   // (16 waves: spills at 128 VGPRs)
  return nullptr;
}

static kfn_t pick_kernel(int nw, int maxacc, int gs) {
  if (gs) return nw == 16 ? pick_acc<16, true>(maxacc) : nullptr;   // global-slot programs: 16 waves
  switch (nw) {
    case 4: return pick_acc<4, false>(maxacc);
    case 8: return pick_acc<8, false>(maxacc);
    case 12: return pick_acc<12, false>(maxacc);
    case 16: return pick_acc<16, false>(maxacc);
    default: return nullptr;
  }
}

static int lds_bytes_of(const int* hdr) {
  return hdr[H_GSLOTS] ? 64 * 4 : (hdr[H_LDS_FLOATS] + 32) * 4;
}

extern "C" int hpe_program_create(const int32_t* words, int64_t n_words, hpe_program** out) {
  if (!words || !out || n_words < H_WORDS) return fail(HPE_EINVAL, "program: null or short word stream");
  if (words[H_MAGIC] != HPE_MAGIC) return fail(HPE_EINVAL, "program: bad magic");
  const int nw = words[H_NW], T = words[H_T];
  const int kind = words[H_KIND];
  const bool fused = kind == KIND_MLP2;
  if (T <= 0 || T % 32) return fail(HPE_EINVAL, "program: T=%d must be a positive multiple of 32", T);
  if (fused && !mlp2_supported(words)) return fail(HPE_EINVAL, "program: unsupported fused 2-layer geometry");
  if (kind == KIND_CHAIN && (!chain_supported(words) || words[H_MODE] != MODE_FWD))
    return fail(HPE_EINVAL, "program: unsupported fused chain geometry");
  if (kind == KIND_RES && !res_supported(words)) return fail(HPE_EINVAL, "program: unsupported residual-stack geometry");
  const int gs = words[H_GSLOTS];
  if (kind == KIND_GENERIC && !pick_kernel(nw, words[H_MAXACC], gs)) return fail(HPE_EINVAL, "program: no kernel for NW=%d MAXACC=%d GSLOTS=%d", nw, words[H_MAXACC], gs);
  if (gs && kind != KIND_GENERIC) return fail(HPE_EINVAL, "program: global slots are for generic programs only");
  if (words[H_NPASS] < 0 || words[H_NPASS] > 64 || (words[H_NPASS] > 1 && words[H_MODE] != MODE_TRAIN))
    return fail(HPE_EINVAL, "program: NPASS=%d (multi-pass programs are training programs, <= 64 passes)", words[H_NPASS]);
  if (words[H_MAXTHIN] > MAXTHIN) return fail(HPE_EINVAL, "program: MAXTHIN=%d > %d", words[H_MAXTHIN], MAXTHIN);
  if (!gs && (int64_t)(words[H_LDS_FLOATS] + 32) * 4 > 160 * 1024) return fail(HPE_EINVAL, "program: LDS %d floats exceeds 160 KiB", words[H_LDS_FLOATS]);
  hpe_program* p = new hpe_program();
  memcpy(p->hdr, words, sizeof(p->hdr));
  p->words = new int[n_words];
  memcpy(p->words, words, n_words * sizeof(int32_t));
  p->n_words = n_words;
  p->epoch = 0;
  p->gscr = nullptr;
  p->wsplit = nullptr;
  p->split_tab = nullptr;
  p->n_split_blocks = 0;
  p->scr_done = nullptr;
  p->scr_stream = nullptr;
  p->scr_used = false;
  // inference programs of the generic interpreter: OP_DENSE ops get a split-weight region (device
  // words O_AUX3), filled from the parameters by split_weights_kernel at every hpe_forward
  std::vector<int> dw(words, words + n_words);
  std::vector<int> tab;
  int64_t nsplit = 0;
  if (kind == KIND_GENERIC && words[H_MODE] == MODE_FWD && !words[H_GSLOTS]) {
    for (int i = 0; i < words[H_NOPS]; ++i) {
      const int wo = words[H_OPS_OFF] + i * O_WORDS;
      if (words[wo + O_TYPE] != OP_DENSE) continue;
      const int K = words[wo + O_K], N = words[wo + O_N];
      const int ncb = (N + 31) >> 5, nks = (K + 15) >> 4;
      dw[wo + O_AUX3] = (int)nsplit;
      for (int cb = 0; cb < ncb; ++cb) {
        tab.push_back(wo);
        tab.push_back((int)nsplit);
        tab.push_back(cb);
      }
      nsplit += (int64_t)ncb * nks * 512 + ncb * 32;
    }
  }
  // guard ring (HPE_GUARD_RING words) + the matching "which check fired" words (hpe_guard_peek)
  hipError_t e = hipMalloc(&p->dwords, (n_words + 2 * HPE_GUARD_RING) * sizeof(int32_t));
  if (e != hipSuccess) { delete p; return fail(HPE_ERUNTIME, "hipMalloc: %s", hipGetErrorString(e)); }
  e = hipMemset(p->dwords + n_words, 0, 2 * HPE_GUARD_RING * sizeof(int32_t));
  if (e == hipSuccess) e = hipMemcpy(p->dwords, dw.data(), n_words * sizeof(int32_t), hipMemcpyHostToDevice);
  if (e == hipSuccess && nsplit > 0) {
    e = hipMalloc(&p->wsplit, nsplit * sizeof(float));
    if (e == hipSuccess) e = hipMalloc(&p->split_tab, tab.size() * sizeof(int));
    if (e == hipSuccess) e = hipMemcpy(p->split_tab, tab.data(), tab.size() * sizeof(int), hipMemcpyHostToDevice);
    p->n_split_blocks = (int)(tab.size() / 3);
  }
  if (e != hipSuccess) {
    hipFree(p->dwords); hipFree(p->wsplit); hipFree(p->split_tab); delete[] p->words; delete p;
    return fail(HPE_ERUNTIME, "hipMalloc / hipMemcpy: %s", hipGetErrorString(e));
  }
  int dev = 0;
  hipGetDevice(&dev);
  int ncu = 256;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  p->n_cu = ncu;
  const int lds_bytes = gs ? (160 * 1024) / 2 : (words[H_LDS_FLOATS] + 32) * 4;   // GS: 2 x 16 waves per CU
  int per_cu = (160 * 1024) / (lds_bytes > 0 ? lds_bytes : 1);
  const int by_waves = 32 / nw;
  if (per_cu > by_waves) per_cu = by_waves;
  if (words[H_WG_PER_CU] > 0 && per_cu > words[H_WG_PER_CU]) per_cu = words[H_WG_PER_CU];
  if (per_cu < 1) per_cu = 1;
  p->grid_cap = ncu * per_cu;
  if (fused) {
    p->grid_cap = mlp2_grid_cap(words, ncu);
  } else if (kind == KIND_CHAIN) {
    p->grid_cap = chain_grid_cap(ncu);
  } else if (kind == KIND_RES) {
    p->grid_cap = res_grid_cap(ncu);
  } else {
    kfn_t k = pick_kernel(nw, words[H_MAXACC], gs);
    hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes_of(words));
#ifndef RP_NO_OCC
    // the persistent grid no larger than the workgroups that are resident at once as the runtime
    // counts them (VGPRs + AGPRs of the instantiation, LDS): past that the tiles run in a second round
    int res = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&res, (const void*)k, nw * 64, lds_bytes_of(words)) == hipSuccess &&
        res > 0 && res < per_cu)
      p->grid_cap = ncu * res;
    kfn_t ks = p->wsplit ? pick_split(nw, words[H_MAXACC]) : nullptr;
    if (ks) {
      hipFuncSetAttribute((const void*)ks, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes_of(words));
      res = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&res, (const void*)ks, nw * 64, lds_bytes_of(words)) == hipSuccess &&
          res > 0 && ncu * res < p->grid_cap)
        p->grid_cap = ncu * res;
    }
#endif
    if (gs) {
      e = hipMalloc(&p->gscr, (size_t)p->grid_cap * words[H_LDS_FLOATS] * sizeof(float));
      if (e != hipSuccess) {
        hipFree(p->dwords); delete[] p->words; delete p;
        return fail(HPE_ERUNTIME, "hipMalloc(global slots): %s", hipGetErrorString(e));
      }
    }
  }
  *out = p;
  return HPE_OK;
}

extern "C" int hpe_program_destroy(hpe_program* p) {
  if (!p) return HPE_OK;
  hipFree(p->dwords);
  if (p->gscr) hipFree(p->gscr);
  if (p->wsplit) hipFree(p->wsplit);
  if (p->split_tab) hipFree(p->split_tab);
  if (p->scr_done) hipEventDestroy(p->scr_done);
  delete[] p->words;
  delete p;
  return HPE_OK;
}

extern "C" int hpe_guard_peek(const hpe_program* p, int32_t* out) {
  if (!p || !out) return fail(HPE_EINVAL, "hpe_guard_peek: null argument");
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(out + 1, p->dwords + p->n_words, 2 * HPE_GUARD_RING * sizeof(int32_t), hipMemcpyDeviceToHost));
  out[0] = __atomic_load_n(&p->epoch, __ATOMIC_RELAXED);
  return HPE_OK;
}

extern "C" int hpe_launch_grid(const hpe_program* p, int64_t n_rows) {
  if (!p) return 0;
  int64_t ntiles = (n_rows + p->hdr[H_T] - 1) / p->hdr[H_T];
  if (p->hdr[H_KIND] == KIND_CHAIN) ntiles = (ntiles + p->hdr[H_NW] - 1) / p->hdr[H_NW];  // per-wave tiles
  int64_t g = ntiles < p->grid_cap ? ntiles : p->grid_cap;
  return (int)(g < 1 ? 1 : g);
}

extern "C" size_t hpe_workspace_size(const hpe_program* p, int64_t n_rows) {
  if (!p) return 0;
  return (size_t)hpe_launch_grid(p, n_rows) * p->hdr[H_SLAB] * sizeof(float);
}

static int launch(const hpe_program* p, Args a, int64_t nrows, hipStream_t s) {
  const int grid = hpe_launch_grid(p, nrows);
  // a ring of guard words indexed by the launch epoch: launches of one program in flight on
  // different streams (up to HPE_GUARD_RING at once) never share the word their split kernel sets
  // and their exact kernel reads; the epoch counter is bumped atomically (host threads)
  int ep = __atomic_add_fetch(&p->epoch, 1, __ATOMIC_RELAXED);
  if (ep <= 0) {
    __atomic_store_n(&p->epoch, 1, __ATOMIC_RELAXED);
    ep = 1;
  }
  a.epoch = ep;
  a.guard = p->dwords + p->n_words + (ep % HPE_GUARD_RING);
  if (p->hdr[H_KIND] == KIND_MLP2) {
    if (mlp2_launch(p->words, a, grid, s)) return fail(HPE_ERUNTIME, "mlp2 launch: %s", hipGetErrorString(hipGetLastError()));
    return HPE_OK;
  }
  if (p->hdr[H_KIND] == KIND_CHAIN) {
    if (chain_launch(p->words, a, grid, s)) return fail(HPE_ERUNTIME, "chain launch: %s", hipGetErrorString(hipGetLastError()));
    return HPE_OK;
  }
  if (p->hdr[H_KIND] == KIND_RES) {
    if (res_launch(p->words, a, grid, s)) return fail(HPE_ERUNTIME, "residual-stack launch: %s", hipGetErrorString(hipGetLastError()));
    return HPE_OK;
  }
  kfn_t k = pick_kernel(p->hdr[H_NW], p->hdr[H_MAXACC], p->hdr[H_GSLOTS]);
  a.gscr = p->gscr;
  kfn_t ks = p->wsplit && !hpe_exact_fp32() ? pick_split(p->hdr[H_NW], p->hdr[H_MAXACC]) : nullptr;
  // the program's shared scratch (device-scratch tile slots, split weights): ordered after the
  // previous launch that used it when that launch went to another stream
  std::unique_lock<std::mutex> scr_lock(p->scr_mu, std::defer_lock);
  const bool uses_scr = p->gscr || ks;
  if (uses_scr) {
    scr_lock.lock();
    if (!p->scr_done) HIPCHK(hipEventCreateWithFlags(&p->scr_done, hipEventDisableTiming));
    if (p->scr_used && p->scr_stream != s) HIPCHK(hipStreamWaitEvent(s, p->scr_done, 0));
  }
  struct ScrRecord {  // records scr_done on s once the launches below are queued
    const hpe_program* p;
    hipStream_t s;
    bool on;
    ~ScrRecord() {
      if (on && hipEventRecord(p->scr_done, s) == hipSuccess) {
        p->scr_stream = s;
        p->scr_used = true;
      }
    }
  } scr_rec{p, s, uses_scr};
  if (ks) {
    // split the current weights (one workgroup per 32-column block), the split interpreter, then
    // its exact-fp32 twin, which exits at once unless the split launch flagged a non-finite value
    hipLaunchKernelGGL(split_weights_kernel, dim3(p->n_split_blocks), dim3(256), 0, s, (const int*)p->dwords,
                       (const int*)p->split_tab, a.params, a.params_t, p->wsplit);
    HIPCHK(hipGetLastError());
    a.wsplit = p->wsplit;
    const int tv = hpe_tev_begin(s);
    hipLaunchKernelGGL(ks, dim3(grid), dim3(p->hdr[H_NW] * 64), lds_bytes_of(p->hdr), s, a);
    const hipError_t le = hipGetLastError();
    hpe_tev_end(s, tv);
    HIPCHK(le);
    hipLaunchKernelGGL(k, dim3(grid), dim3(p->hdr[H_NW] * 64), lds_bytes_of(p->hdr), s, a);
    HIPCHK(hipGetLastError());
    return HPE_OK;
  }
  a.guard = nullptr;  // no split launch ahead: the kernel runs unconditionally
  const int npass = p->hdr[H_MODE] == MODE_TRAIN && p->hdr[H_NPASS] > 1 ? p->hdr[H_NPASS] : 1;
  const int tv = hpe_tev_begin(s);
  hipError_t le = hipSuccess;
  for (int pass = 0; pass < npass && le == hipSuccess; ++pass) {
    a.pass = pass;
    hipLaunchKernelGGL(k, dim3(grid), dim3(p->hdr[H_NW] * 64), lds_bytes_of(p->hdr), s, a);
    le = hipGetLastError();
  }
  hpe_tev_end(s, tv);
  HIPCHK(le);
  return HPE_OK;
}

extern "C" int hpe_forward(const hpe_program* p, const float* params, const float* params_t,
                           const float* x, int64_t n_images, int32_t P, const int32_t* idx,
                           float* y, void* stream) {
  if (!p || !params || !x || !y) return fail(HPE_EINVAL, "hpe_forward: null argument");
  if (p->hdr[H_MODE] != MODE_FWD) return fail(HPE_EINVAL, "hpe_forward: program not compiled for inference");
  if (n_images < 0 || P <= 0) return fail(HPE_EINVAL, "hpe_forward: bad shape n_images=%lld P=%d", (long long)n_images, P);
  if (n_images == 0) return HPE_OK;
  Args a = {};
  a.prog = p->dwords; a.params = params; a.params_t = params_t ? params_t : params; a.x = x;
  a.idx = idx; a.y = y; a.nrows = n_images * (int64_t)P; a.P = P;
  return launch(p, a, a.nrows, (hipStream_t)stream);
}

extern "C" int hpe_train_step_bounded(const hpe_program* p, const float* params, const float* params_t,
                                      const float* x, const float* ytrue, int64_t n_images, int32_t P,
                                      const int32_t* idx, int64_t img_off, float inv_count, uint64_t seed,
                                      float x_bound, void* ws, void* stream) {
  if (!p || !params || !x || !ytrue || !ws) return fail(HPE_EINVAL, "hpe_train_step: null argument");
  if (!(x_bound >= 0.f)) return fail(HPE_EINVAL, "hpe_train_step_bounded: bad bound");
  if (p->hdr[H_MODE] == MODE_FWD) return fail(HPE_EINVAL, "hpe_train_step: program compiled for inference only");
  if (n_images <= 0 || P <= 0) return fail(HPE_EINVAL, "hpe_train_step: bad shape n_images=%lld P=%d", (long long)n_images, P);
  Args a = {};
  a.prog = p->dwords; a.params = params; a.params_t = params_t ? params_t : params; a.x = x;
  a.ytrue = ytrue; a.idx = idx; a.ws = (float*)ws; a.nrows = n_images * (int64_t)P; a.P = P;
  a.img_off = img_off; a.inv_count = inv_count; a.seed = seed; a.x_bound = x_bound;
  return launch(p, a, a.nrows, (hipStream_t)stream);
}

extern "C" int hpe_train_step(const hpe_program* p, const float* params, const float* params_t,
                              const float* x, const float* ytrue, int64_t n_images, int32_t P,
                              const int32_t* idx, int64_t img_off, float inv_count, uint64_t seed,
                              void* ws, void* stream) {
  if (!p || !params || !x || !ytrue || !ws) return fail(HPE_EINVAL, "hpe_train_step: null argument");
  if (p->hdr[H_MODE] == MODE_FWD) return fail(HPE_EINVAL, "hpe_train_step: program compiled for inference only");
  if (n_images <= 0 || P <= 0) return fail(HPE_EINVAL, "hpe_train_step: bad shape n_images=%lld P=%d", (long long)n_images, P);
  Args a = {};
  a.prog = p->dwords; a.params = params; a.params_t = params_t ? params_t : params; a.x = x;
  a.ytrue = ytrue; a.idx = idx; a.ws = (float*)ws; a.nrows = n_images * (int64_t)P; a.P = P;
  a.img_off = img_off; a.inv_count = inv_count; a.seed = seed;
  return launch(p, a, a.nrows, (hipStream_t)stream);
}

extern "C" int hpe_reduce(const hpe_program* p, int64_t n_rows, const void* ws, float* grad, void* stream) {
  if (!p || !ws || !grad) return fail(HPE_EINVAL, "hpe_reduce: null argument");
  const int grid = hpe_launch_grid(p, n_rows);
  const int n = p->hdr[H_NPARAMS_TRAIN] + 4;
  hipLaunchKernelGGL(reduce_kernel, dim3((n + 63) / 64), dim3(256), 0, (hipStream_t)stream,
                     (const float*)ws, grad, grid, p->hdr[H_SLAB], n);
  HIPCHK(hipGetLastError());
  return HPE_OK;
}

extern "C" int hpe_optim_grid(int64_t n) {
  int64_t g = (n + 255) / 256;
  if (g > 1024) g = 1024;
  return (int)(g < 1 ? 1 : g);
}

extern "C" int hpe_optim_step(int32_t kind, float lr, float b1, float b2, float eps, int64_t iter,
                              float gscale, float* w, float* wt, float* m, float* v,
                              const float* grad, const float* l2, const int32_t* tpos, int64_t n,
                              float* regp, void* stream) {
  if (!w || !grad || !l2 || !tpos || !regp) return fail(HPE_EINVAL, "hpe_optim_step: null argument");
  if (kind != HPE_OPT_SGD && (!m || !v)) return fail(HPE_EINVAL, "hpe_optim_step: Adam/Adamax need m and v");
  if (iter < 1) return fail(HPE_EINVAL, "hpe_optim_step: iter must be >= 1");
  double alpha = lr;
  if (kind == HPE_OPT_ADAM) {
    const double b1p = pow((double)b1, (double)iter), b2p = pow((double)b2, (double)iter);
    alpha = (double)lr * sqrt(1.0 - b2p) / (1.0 - b1p);
  } else if (kind == HPE_OPT_ADAMAX) {
    alpha = (double)lr / (1.0 - pow((double)b1, (double)iter));
  } else if (kind != HPE_OPT_SGD) {
    return fail(HPE_EINVAL, "hpe_optim_step: unknown optimizer kind %d", kind);
  }
  const int grid = hpe_optim_grid(n);
  hipLaunchKernelGGL(optim_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, kind, lr,
                     (float)alpha, b1, b2, eps, gscale, w, wt ? wt : w, m, v, grad, l2, tpos, n, regp);
  HIPCHK(hipGetLastError());
  return HPE_OK;
}

extern "C" int hpe_reduce_optim_step(const hpe_program* p, int64_t n_rows, const void* ws, float* grad,
                                     int32_t kind, float lr, float b1, float b2, float eps, int64_t iter,
                                     float gscale, float* w, float* wt, float* m, float* v, const float* l2,
                                     const int32_t* tpos, int64_t n, float* regp, void* stream) {
  if (!p || !ws || !grad || !w || !l2 || !tpos || !regp) return fail(HPE_EINVAL, "hpe_reduce_optim_step: null argument");
  if (n != p->hdr[H_NPARAMS_TRAIN])
    return fail(HPE_EINVAL, "hpe_reduce_optim_step: n = %lld, the program trains %d parameters", (long long)n,
                p->hdr[H_NPARAMS_TRAIN]);
  if (kind != HPE_OPT_SGD && (!m || !v)) return fail(HPE_EINVAL, "hpe_reduce_optim_step: Adam/Adamax need m and v");
  if (iter < 1) return fail(HPE_EINVAL, "hpe_reduce_optim_step: iter must be >= 1");
  double alpha = lr;
  if (kind == HPE_OPT_ADAM) {
    const double b1p = pow((double)b1, (double)iter), b2p = pow((double)b2, (double)iter);
    alpha = (double)lr * sqrt(1.0 - b2p) / (1.0 - b1p);
  } else if (kind == HPE_OPT_ADAMAX) {
    alpha = (double)lr / (1.0 - pow((double)b1, (double)iter));
  } else if (kind != HPE_OPT_SGD) {
    return fail(HPE_EINVAL, "hpe_reduce_optim_step: unknown optimizer kind %d", kind);
  }
  const int sgrid = hpe_launch_grid(p, n_rows);
  const int grid = hpe_optim_grid(n);
  hipLaunchKernelGGL(reduce_optim_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const float*)ws, sgrid,
                     p->hdr[H_SLAB], kind, lr, (float)alpha, b1, b2, eps, gscale, w, wt ? wt : w, m, v, grad, l2,
                     tpos, n, regp);
  HIPCHK(hipGetLastError());
  return HPE_OK;
}

// ---- hpe_fit_steps: fit's per-step path for one epoch, the step loop in C -----------------------
// The launches fit's Python loop issues per step, in the same order with the same arguments (so the
// results are bit-identical), without a Python round trip per step: hpe_train_step_bounded, then
// hpe_reduce_optim_step when the launch grid is small (single rank) or hpe_reduce + hpe_optim_step.
#define HPE_FUSED_REDUCE_MAX_GRID 16   // hpe/engine.py Engine.FUSED_REDUCE_MAX_GRID
extern "C" int hpe_fit_steps(const hpe_program* p, float* params, float* params_t, float* m, float* v,
                             const float* l2, const int32_t* tpos, int64_t n_train, const float* x,
                             const float* ytrue, const int32_t* perm, int64_t n, int32_t batch, int32_t P,
                             float x_bound, int32_t kind, float lr, float b1, float b2, float eps,
                             uint64_t seed_base, int64_t iter0, void* ws, float* grad, float* stats,
                             int32_t stats_stride, void* stream) {
  if (!p || !params || !x || !ytrue || !perm || !ws || !grad || !l2 || !tpos || !stats)
    return fail(HPE_EINVAL, "hpe_fit_steps: null argument");
  if (n <= 0 || batch <= 0 || P <= 0 || iter0 < 0)
    return fail(HPE_EINVAL, "hpe_fit_steps: bad shape n=%lld batch=%d P=%d", (long long)n, batch, P);
  if (n_train != p->hdr[H_NPARAMS_TRAIN]) return fail(HPE_EINVAL, "hpe_fit_steps: n_train mismatch");
  // every step's optimizer launch writes stats row s: [sse, sae, reg_0 .. reg_{grid-1}]
  if ((int64_t)stats_stride < 2 + (int64_t)hpe_optim_grid(n_train))
    return fail(HPE_EINVAL, "hpe_fit_steps: stats_stride %d < 2 + hpe_optim_grid(n_train) = %d", stats_stride,
                2 + hpe_optim_grid(n_train));
  const int64_t steps = (n + batch - 1) / batch;
  for (int64_t s = 0; s < steps; ++s) {
    const int64_t b0 = s * batch, nb = (n - b0) < batch ? (n - b0) : batch;
    const int64_t rows = nb * P, it = iter0 + 1 + s;
    // inv_count as fit computes it: 1 / (nb P 3) in double, rounded to float
    const float inv = (float)(1.0 / (double)(rows * 3));
    int rc = hpe_train_step_bounded(p, params, params_t, x, ytrue, nb, P, perm + b0, 0, inv, seed_base + (uint64_t)it,
                                    x_bound, ws, stream);
    if (rc) return rc;
    float* st = stats + s * stats_stride;
    if (hpe_launch_grid(p, rows) <= HPE_FUSED_REDUCE_MAX_GRID) {
      rc = hpe_reduce_optim_step(p, rows, ws, grad, kind, lr, b1, b2, eps, it, 1.f, params, params_t, m, v, l2, tpos,
                                 n_train, st, stream);
    } else {
      rc = hpe_reduce(p, rows, ws, grad, stream);
      if (!rc) rc = hpe_optim_step(kind, lr, b1, b2, eps, it, 1.f, params, params_t, m, v, grad, l2, tpos, n_train, st, stream);
    }
    if (rc) return rc;
  }
  return HPE_OK;
}

// ---- hpe_fit_steps_dp: the same step loop for one rank of a data-parallel fit ------------------
// Per step, the launches fit's data-parallel Python loop issues (hpe/model.py): this rank's
// contiguous share [r0, r1) of the global batch (hpe.parallel.batch_slice), hpe_train_step_bounded
// with img_off = r0 - b0 and the GLOBAL element count, hpe_reduce (or a zeroed gradient for an empty
// share), the caller's all-reduce of [gradient | sse, sae, 0, 0], then hpe_optim_step — no Python
// round trip per step besides the all-reduce hook itself.
extern "C" int hpe_fit_steps_dp(const hpe_program* p, float* params, float* params_t, float* m, float* v,
                                const float* l2, const int32_t* tpos, int64_t n_train, const float* x,
                                const float* ytrue, const int32_t* perm, int64_t n, int32_t batch, int32_t P,
                                float x_bound, int32_t kind, float lr, float b1, float b2, float eps,
                                uint64_t seed_base, int64_t iter0, void* ws, float* grad, float* stats,
                                int32_t stats_stride, int32_t rank, int32_t world, hpe_allreduce_fn allreduce,
                                void* user, int64_t* steps_done, void* stream) {
  if (steps_done) *steps_done = 0;
  if (!p || !params || !x || !ytrue || !perm || !ws || !grad || !l2 || !tpos || !stats || !allreduce)
    return fail(HPE_EINVAL, "hpe_fit_steps_dp: null argument");
  if (n <= 0 || batch <= 0 || P <= 0 || iter0 < 0 || world < 1 || rank < 0 || rank >= world)
    return fail(HPE_EINVAL, "hpe_fit_steps_dp: bad shape n=%lld batch=%d P=%d rank=%d world=%d", (long long)n, batch,
                P, rank, world);
  if (n_train != p->hdr[H_NPARAMS_TRAIN]) return fail(HPE_EINVAL, "hpe_fit_steps_dp: n_train mismatch");
  if ((int64_t)stats_stride < 2 + (int64_t)hpe_optim_grid(n_train))
    return fail(HPE_EINVAL, "hpe_fit_steps_dp: stats_stride %d < 2 + hpe_optim_grid(n_train) = %d", stats_stride,
                2 + hpe_optim_grid(n_train));
  hipStream_t s = (hipStream_t)stream;
  const int64_t steps = (n + batch - 1) / batch;
  for (int64_t st = 0; st < steps; ++st) {
    const int64_t b0 = st * batch, nb = (n - b0) < batch ? (n - b0) : batch;
    const int64_t r0 = b0 + (nb * rank) / world, r1 = b0 + (nb * (rank + 1)) / world;
    const int64_t it = iter0 + 1 + st;
    const float inv = (float)(1.0 / (double)(nb * P * 3));
    int rc;
    if (r1 > r0) {
      rc = hpe_train_step_bounded(p, params, params_t, x, ytrue, r1 - r0, P, perm + r0, r0 - b0, inv,
                                  seed_base + (uint64_t)it, x_bound, ws, stream);
      if (!rc) rc = hpe_reduce(p, (r1 - r0) * P, ws, grad, stream);
    } else {
      rc = hipMemsetAsync(grad, 0, (n_train + 4) * sizeof(float), s) == hipSuccess
               ? HPE_OK : fail(HPE_ERUNTIME, "hpe_fit_steps_dp: memset");
    }
    if (rc) return rc;
    if (allreduce(grad, n_train + 4, stream, user) != 0)
      return fail(HPE_ERUNTIME, "hpe_fit_steps_dp: all-reduce hook failed at step %lld", (long long)st);
    rc = hpe_optim_step(kind, lr, b1, b2, eps, it, 1.f, params, params_t, m, v, grad, l2, tpos, n_train,
                        stats + st * stats_stride, stream);
    if (rc) return rc;
    if (steps_done) *steps_done = st + 1;  // optimizer steps applied: the caller's iteration count
  }
  return HPE_OK;
}
