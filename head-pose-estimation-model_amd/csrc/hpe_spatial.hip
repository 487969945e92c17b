// hpe_spatial.hip — the two non-row-local stages of the reference's attention heads on H x W > 1
// feature maps (Model-88/attention_model.py:16-72 se_transformer_regr_head
// and :74-90 create_modelC, applied to a BlazeFace tap such as re_lu_10 16x16x88):
//
//   hpe_se_gate  SE channel gating per image (attention_model.py:34-38):
//                s = act2(W2 . act1(W1 . mean_HW(x) + b1) + b2);  xg = x * s   (broadcast over H,W)
//                one workgroup per image: fixed-order mean (deterministic), the two tiny dense
//                layers in LDS, then the gated rows (the image's second read hits L2)
//   hpe_mha      the self-attention core of MultiHeadAttention over the H*W tokens of each image
//                (attention_model.py:52-55, Keras MHA with attention_axes [1]):
//                o_h = softmax(q_h k_h^T) v_h per head, q pre-scaled by 1/sqrt(key_dim)
//                one workgroup per (image, head, 256 queries), one query per thread; keys / values
//                of the head stream through LDS in blocks of 256 tokens; online softmax over
//                32-key sub-blocks (one max + 32 exps per sub-block, fp32 throughout)
//
//   hpe_seg_mean per-image mean of rows: a terminal GlobalAveragePooling2D (Flatten-era graphs)
//
// The row-local parts (Q/K/V and output projections, residual adds, LayerNorms, feed-forward and
// the 1x1-conv regressor) run as ordinary row programs (hpe/spatial.py builds them).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/hpe.h"
#include "hpe_common.h"

#define SE_NT 256
#define SE_MAXC 512
#define SE_MAXU 512

__global__ void __launch_bounds__(SE_NT) se_gate_kernel(const float* __restrict__ x, float* __restrict__ xg,
                                                        int P, int C, const float* __restrict__ w1,
                                                        const float* __restrict__ b1, int U, int act1,
                                                        const float* __restrict__ w2,
                                                        const float* __restrict__ b2, int act2) {
  __shared__ float part[SE_NT * 4];
  __shared__ float mean[SE_MAXC];
  __shared__ float hid[SE_MAXU];
  __shared__ float gate[SE_MAXC];
  const int t = threadIdx.x;
  const int64_t base = (int64_t)blockIdx.x * P * C;
  // ---- mean over the P rows: thread -> (channel quad q, row phase ro), fixed-order combine ----
  const int C4 = C >> 2;
  const int RS = SE_NT / C4;             // row phases (threads >= RS * C4 idle)
  const int q = t % C4, ro = t / C4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (ro < RS)
    for (int r = ro; r < P; r += RS) acc += *(const f32x4*)(x + base + (int64_t)r * C + 4 * q);
  *(f32x4*)(part + 4 * t) = acc;
  __syncthreads();
  if (t < C4) {
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    for (int p = 0; p < RS; ++p) s += *(const f32x4*)(part + 4 * (p * C4 + t));
    const float inv = 1.f / (float)P;
    mean[4 * t + 0] = s.x * inv;
    mean[4 * t + 1] = s.y * inv;
    mean[4 * t + 2] = s.z * inv;
    mean[4 * t + 3] = s.w * inv;
  }
  __syncthreads();
  // ---- squeeze / excite ----
  for (int u = t; u < U; u += SE_NT) {
    float z = b1 ? b1[u] : 0.f;
    for (int c = 0; c < C; ++c) z = fmaf(mean[c], w1[(int64_t)c * U + u], z);
    hid[u] = act_f(act1, z);
  }
  __syncthreads();
  for (int c = t; c < C; c += SE_NT) {
    float z = b2 ? b2[c] : 0.f;
    for (int u = 0; u < U; ++u) z = fmaf(hid[u], w2[(int64_t)u * C + c], z);
    gate[c] = act_f(act2, z);
  }
  __syncthreads();
  // ---- gated rows ----
  const int64_t nq = (int64_t)P * C4;
  for (int64_t e = t; e < nq; e += SE_NT) {
    const int64_t r = e / C4;
    const int qq = (int)(e - r * C4);
    const f32x4 g = *(const f32x4*)(gate + 4 * qq);
    *(f32x4*)(xg + base + r * C + 4 * qq) = *(const f32x4*)(x + base + r * C + 4 * qq) * g;
  }
}

// per-image mean of the rows: the GlobalAveragePooling2D that ends the Flatten-era Model-96 graphs
// (create_model -> GAP, e.g. checkpoint nkjq2rpb) on H x W > 1 maps; fixed order, deterministic
__global__ void __launch_bounds__(SE_NT) seg_mean_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                         int P, int C) {
  __shared__ float part[SE_NT];
  const int t = threadIdx.x;
  const int RS = SE_NT / C;  // row phases per channel
  const int c = t % C, ro = t / C;
  const float* xi = x + (int64_t)blockIdx.x * P * C;
  float acc = 0.f;
  if (ro < RS)
    for (int r = ro; r < P; r += RS) acc += xi[(int64_t)r * C + c];
  part[t] = acc;
  __syncthreads();
  if (t < C) {
    float s = 0.f;
    for (int p = 0; p < RS; ++p) s += part[p * C + t];
    y[(int64_t)blockIdx.x * C + t] = s / (float)P;
  }
}

// rows in: [pass-through (C) | q (H*D) | k (H*D) | v (H*D)], stride ld_in
// rows out: [pass-through (C) | o (H*D)], stride ld_out (the pass-through copy by head 0 only)
#define MHA_QB 256   // queries per workgroup (one per thread)
#define MHA_KB 256   // keys per LDS block
#define MHA_SB 32    // keys per online-softmax sub-block

// D: key_dim padded to a multiple of 4 (zero lanes past KD, the real key_dim)
template <int D>
__global__ void __launch_bounds__(MHA_QB) mha_kernel(const float* __restrict__ in, int ld_in, int C, int qoff,
                                                     const float* __restrict__ ps, int ld_ps,
                                                     float* __restrict__ out, int ld_out, int P, int H,
                                                     int nqb, int KD) {
  __shared__ __attribute__((aligned(16))) float ks[MHA_KB * D];
  __shared__ __attribute__((aligned(16))) float vs[MHA_KB * D];
  const int t = threadIdx.x;
  const int qb = blockIdx.x % nqb;
  const int h = (blockIdx.x / nqb) % H;
  const int64_t img = blockIdx.x / (nqb * H);
  const int HD = H * KD;
  const int64_t row0 = img * P;
  const int qi = qb * MHA_QB + t;
  const bool qok = qi < P;
  const float* qrow = in + (row0 + (qok ? qi : 0)) * ld_in;
  float qv[D], o[D];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    qv[d] = d < KD ? qrow[qoff + h * KD + d] : 0.f;
    o[d] = 0.f;
  }
  float m = -INFINITY, l = 0.f;
  for (int k0 = 0; k0 < P; k0 += MHA_KB) {
    const int nk = min(MHA_KB, P - k0);
    __syncthreads();  // previous block's readers are done
    for (int e = t; e < nk * D; e += MHA_QB) {
      const int j = e / D, d = e - j * D;
      const float* kr = in + (row0 + k0 + j) * ld_in + qoff + HD + h * KD;
      ks[e] = d < KD ? kr[d] : 0.f;
      vs[e] = d < KD ? kr[HD + d] : 0.f;
    }
    __syncthreads();
    for (int j0 = 0; j0 < nk; j0 += MHA_SB) {
      const int nj = min(MHA_SB, nk - j0);
      float s[MHA_SB];
      float mb = -INFINITY;
#pragma unroll
      for (int j = 0; j < MHA_SB; ++j) {
        float a = 0.f;
        if (j < nj) {
          const float* kr = ks + (j0 + j) * D;
#pragma unroll
          for (int d = 0; d < D; d += 4) {
            const f32x4 kk = *(const f32x4*)(kr + d);
            a = fmaf(qv[d], kk.x, a);
            a = fmaf(qv[d + 1], kk.y, a);
            a = fmaf(qv[d + 2], kk.z, a);
            a = fmaf(qv[d + 3], kk.w, a);
          }
          mb = fmaxf(mb, a);
        }
        s[j] = a;
      }
      const float mn = fmaxf(m, mb);
      const float corr = __expf(m - mn);  // m = -inf on the first sub-block -> 0
      l *= corr;
#pragma unroll
      for (int d = 0; d < D; ++d) o[d] *= corr;
#pragma unroll
      for (int j = 0; j < MHA_SB; ++j) {
        if (j < nj) {
          const float p = __expf(s[j] - mn);
          l += p;
          const float* vr = vs + (j0 + j) * D;
#pragma unroll
          for (int d = 0; d < D; d += 4) {
            const f32x4 vv = *(const f32x4*)(vr + d);
            o[d] = fmaf(p, vv.x, o[d]);
            o[d + 1] = fmaf(p, vv.y, o[d + 1]);
            o[d + 2] = fmaf(p, vv.z, o[d + 2]);
            o[d + 3] = fmaf(p, vv.w, o[d + 3]);
          }
        }
      }
      m = mn;
    }
  }
  if (!qok) return;
  const float inv = 1.f / l;
  float* orow = out + (row0 + qi) * ld_out;
#pragma unroll
  for (int d = 0; d < D; ++d)
    if (d < KD) orow[C + h * KD + d] = o[d] * inv;
  if (h == 0)
    for (int c = 0; c < C; ++c) orow[c] = ps[(row0 + qi) * ld_ps + c];
}


// ------------------------------------------------------------------------------------------------
// hpe_mha on fp32 MFMA (key_dim <= 32, every checkpoint but none): flash-style, one wave per 32
// queries, exact fp32 (v_mfma_f32_32x32x2_f32), keys / values of the head streamed through LDS in
// blocks of MHAM_KB tokens, 32-key sub-blocks:
//   S^T[key i][query j] = K_blk . Q^T  (A = K rows from LDS, lane = key; B = Q^T from the wave's
//                                       registers, lane = query)  -> accumulator: lane = query j,
//                                       16 registers = keys (g & 3) + 8 (g >> 2) + 4 half
//   online softmax per query: the 32 scores of a sub-block sit in lanes j and j + 32 (one xor-32
//   exchange for the max); each lane keeps its own partial exp-sum (combined once at the end)
//   O^T[d][query j] += V^T . P^T  (B = P^T is the score accumulator itself: MFMA step t takes
//                                   register t, i.e. key (t & 3) + 8 (t >> 2) + 4 half on half h;
//                                   A = V^T, lane = d, read from LDS for that same key)
//   -> O^T accumulator: lane = query j, registers = d rows: the output row of query j, no shuffles.
// The VALU kernel above remains for key_dim > 32.
// ------------------------------------------------------------------------------------------------
#define MHAM_W 4              // waves per workgroup (32 queries each)
#define MHAM_KB 128           // keys per LDS block
template <int D>              // key_dim padded to an even number <= 32
__global__ void __launch_bounds__(MHAM_W * 64) mha_mfma_kernel(const float* __restrict__ in, int ld_in, int C, int qoff,
                                                               const float* __restrict__ ps, int ld_ps,
                                                               float* __restrict__ out, int ld_out, int P, int H,
                                                               int nqb, int KD) {
  constexpr int DS = D + 1;   // LDS row stride (odd: the 32 key rows of an A read hit distinct banks)
  __shared__ float ks[MHAM_KB * DS];
  __shared__ float vs[MHAM_KB * DS];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, half = lane >> 5, l32 = lane & 31;
  const int qb = blockIdx.x % nqb;
  const int h = (blockIdx.x / nqb) % H;
  const int64_t img = blockIdx.x / (nqb * H);
  const int HD = H * KD;
  const int64_t row0 = img * P;
  const int q = qb * (MHAM_W * 32) + wave * 32 + l32;   // this lane's query (both halves)
  const bool qok = q < P;
  // Q^T operand of step t: Q[q][2t + half]
  float qv[D / 2];
  {
    const float* qr = in + (row0 + (qok ? q : 0)) * ld_in + qoff + h * KD;
#pragma unroll
    for (int t = 0; t < D / 2; ++t) {
      const int d = 2 * t + half;
      qv[t] = (qok && d < KD) ? qr[d] : 0.f;
    }
  }
  f32x16 o = {};
  float m = -INFINITY, l = 0.f;
  for (int k0 = 0; k0 < P; k0 += MHAM_KB) {
    const int nk = min(MHAM_KB, P - k0);
    __syncthreads();  // the previous block's readers are done
    for (int e = threadIdx.x; e < MHAM_KB * D; e += MHAM_W * 64) {
      const int j = e / D, d = e - j * D;
      float kv = 0.f, vv = 0.f;
      if (j < nk && d < KD) {
        const float* kr = in + (row0 + k0 + j) * ld_in + qoff + HD + h * KD;
        kv = kr[d];
        vv = kr[HD + d];
      }
      ks[j * DS + d] = kv;
      vs[j * DS + d] = vv;
    }
    __syncthreads();
    for (int j0 = 0; j0 < nk; j0 += 32) {
      // S^T block: A = K rows j0 + l32 (lane = key), k = 2t + half
      f32x16 sacc = {};
      const float* kr = ks + (j0 + l32) * DS + half;
#pragma unroll
      for (int t = 0; t < D / 2; ++t) sacc = __builtin_amdgcn_mfma_f32_32x32x2f32(kr[2 * t], qv[t], sacc, 0, 0, 0);
      // keys past the block end: -inf (exp -> 0)
      float mb = -INFINITY;
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int key = j0 + (g & 3) + 8 * (g >> 2) + 4 * half;
        if (key >= nk) sacc[g] = -INFINITY;
        mb = fmaxf(mb, sacc[g]);
      }
      mb = fmaxf(mb, __shfl_xor(mb, 32, 64));
      const float mn = fmaxf(m, mb);
      const float corr = __expf(m - mn);  // m = -inf on the first sub-block -> 0
      l *= corr;
#pragma unroll
      for (int g = 0; g < 16; ++g) o[g] *= corr;
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        sacc[g] = __expf(sacc[g] - mn);
        l += sacc[g];
      }
      m = mn;
      // O^T += V^T . P^T: step t takes P^T from score register t (key (t&3) + 8(t>>2) + 4 half)
      const float* vr = vs + j0 * DS + (l32 < D ? l32 : 0);
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const int key = (t & 3) + 8 * (t >> 2) + 4 * half;
        const float a = l32 < D ? vr[key * DS] : 0.f;
        o = __builtin_amdgcn_mfma_f32_32x32x2f32(a, sacc[t], o, 0, 0, 0);
      }
    }
  }
  // both halves hold partial exp-sums of their keys
  l += __shfl_xor(l, 32, 64);
  if (qok) {
    const float inv = 1.f / l;
    float* orow = out + (row0 + q) * ld_out + C + h * KD;
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const int d = (g & 3) + 8 * (g >> 2) + 4 * half;
      if (d < KD) orow[d] = o[g] * inv;
    }
  }
  // pass-through columns [0, C) of this workgroup's query rows, by head 0 (coalesced)
  if (h == 0) {
    const int qa = qb * (MHAM_W * 32), qe = min(qa + MHAM_W * 32, P);
    for (int e = threadIdx.x; e < (qe - qa) * C; e += MHAM_W * 64) {
      const int r = e / C, c = e - r * C;
      out[(row0 + qa + r) * ld_out + c] = ps[(row0 + qa + r) * ld_ps + c];
    }
  }
}

extern "C" int hpe_se_gate(const float* x, float* xg, int64_t n_images, int32_t P, int32_t C,
                           const float* w1, const float* b1, int32_t U, int32_t act1, const float* w2,
                           const float* b2, int32_t act2, void* stream) {
  if (!x || !xg || !w1 || !w2) return hpe_fail(HPE_EINVAL, "hpe_se_gate: null argument");
  if (n_images < 0 || P <= 0 || C <= 0 || (C & 3) || C > SE_MAXC || U <= 0 || U > SE_MAXU || C / 4 > SE_NT)
    return hpe_fail(HPE_EINVAL, "hpe_se_gate: unsupported shape P=%d C=%d U=%d", P, C, U);
  if (act1 < 0 || act1 > ACT_LEAKY_RELU || act2 < 0 || act2 > ACT_LEAKY_RELU || act1 == ACT_SWISH || act2 == ACT_SWISH)
    return hpe_fail(HPE_EINVAL, "hpe_se_gate: unsupported activation");
  if (n_images == 0) return HPE_OK;
  hipLaunchKernelGGL(se_gate_kernel, dim3((unsigned)n_images), dim3(SE_NT), 0, (hipStream_t)stream,
                     x, xg, P, C, w1, b1, U, act1, w2, b2, act2);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? HPE_OK : hpe_fail(HPE_ERUNTIME, "hpe_se_gate: %s", hipGetErrorString(e));
}

extern "C" int hpe_seg_mean(const float* x, float* y, int64_t n_images, int32_t P, int32_t C, void* stream) {
  if (!x || !y) return hpe_fail(HPE_EINVAL, "hpe_seg_mean: null argument");
  if (n_images < 0 || P <= 0 || C <= 0 || C > SE_NT) return hpe_fail(HPE_EINVAL, "hpe_seg_mean: bad shape P=%d C=%d", P, C);
  if (n_images == 0) return HPE_OK;
  hipLaunchKernelGGL(seg_mean_kernel, dim3((unsigned)n_images), dim3(SE_NT), 0, (hipStream_t)stream, x, y, P, C);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? HPE_OK : hpe_fail(HPE_ERUNTIME, "hpe_seg_mean: %s", hipGetErrorString(e));
}

// in rows: q at float offset qoff, then k, v; pass-through rows ps (stride ld_ps) -> out[:, :C]
static int mha_launch(const float* in, int32_t ld_in, int32_t qoff, const float* ps, int32_t ld_ps, int32_t C,
                      float* out, int32_t ld_out, int64_t n_images, int32_t P, int32_t H, int32_t D, void* stream) {
  if (n_images == 0) return HPE_OK;
  hipStream_t s = (hipStream_t)stream;
  if (D <= 32 && !getenv("HPE_MHA_VALU")) {
    const int nqb = (P + MHAM_W * 32 - 1) / (MHAM_W * 32);
    const int64_t grid = n_images * H * nqb;
    if (grid > 0x7fffffff) return hpe_fail(HPE_EINVAL, "hpe_mha: grid too large");
#define MHAM_CASE(DD) \
    case DD: hipLaunchKernelGGL(mha_mfma_kernel<DD>, dim3((unsigned)grid), dim3(MHAM_W * 64), 0, s, in, ld_in, C, qoff, ps, ld_ps, out, ld_out, P, H, nqb, D); break;
    switch ((D + 1) & ~1) {
      MHAM_CASE(2) MHAM_CASE(4) MHAM_CASE(6) MHAM_CASE(8) MHAM_CASE(10) MHAM_CASE(12) MHAM_CASE(14) MHAM_CASE(16)
      MHAM_CASE(18) MHAM_CASE(20) MHAM_CASE(22) MHAM_CASE(24) MHAM_CASE(26) MHAM_CASE(28) MHAM_CASE(30) MHAM_CASE(32)
      default: return hpe_fail(HPE_EINVAL, "hpe_mha: key_dim %d", D);
    }
#undef MHAM_CASE
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? HPE_OK : hpe_fail(HPE_ERUNTIME, "hpe_mha: %s", hipGetErrorString(e));
  }
  const int nqb = (P + MHA_QB - 1) / MHA_QB;
  const int64_t grid = n_images * H * nqb;
  if (grid > 0x7fffffff) return hpe_fail(HPE_EINVAL, "hpe_mha: grid too large");
#define MHA_CASE(DD) \
  case DD: hipLaunchKernelGGL(mha_kernel<DD>, dim3((unsigned)grid), dim3(MHA_QB), 0, s, in, ld_in, C, qoff, ps, ld_ps, out, ld_out, P, H, nqb, D); break;
  switch ((D + 3) & ~3) {
    MHA_CASE(4)
    MHA_CASE(8)
    MHA_CASE(12)
    MHA_CASE(16)
    MHA_CASE(24)
    MHA_CASE(32)
    MHA_CASE(48)
    MHA_CASE(64)
    default: return hpe_fail(HPE_EINVAL, "hpe_mha: key_dim %d > 64 or unsupported", D);
  }
#undef MHA_CASE
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? HPE_OK : hpe_fail(HPE_ERUNTIME, "hpe_mha: %s", hipGetErrorString(e));
}

extern "C" int hpe_mha(const float* in, int32_t ld_in, int32_t C, float* out, int32_t ld_out,
                       int64_t n_images, int32_t P, int32_t H, int32_t D, void* stream) {
  if (!in || !out) return hpe_fail(HPE_EINVAL, "hpe_mha: null argument");
  if (n_images < 0 || P <= 0 || C < 0 || H <= 0 || D <= 0 || ld_in < C + 3 * H * D || ld_out < C + H * D)
    return hpe_fail(HPE_EINVAL, "hpe_mha: bad shape P=%d C=%d H=%d D=%d ld_in=%d ld_out=%d", P, C, H, D,
                    ld_in, ld_out);
  return mha_launch(in, ld_in, C, in, ld_in, C, out, ld_out, n_images, P, H, D, stream);
}

extern "C" int hpe_mha_xg(const float* qkv, int32_t ld_qkv, const float* xg, int32_t C, float* out, int32_t ld_out,
                          int64_t n_images, int32_t P, int32_t H, int32_t D, void* stream) {
  if (!qkv || !out || (C > 0 && !xg)) return hpe_fail(HPE_EINVAL, "hpe_mha_xg: null argument");
  if (n_images < 0 || P <= 0 || C < 0 || H <= 0 || D <= 0 || ld_qkv < 3 * H * D || ld_out < C + H * D)
    return hpe_fail(HPE_EINVAL, "hpe_mha_xg: bad shape P=%d C=%d H=%d D=%d ld_qkv=%d ld_out=%d", P, C, H, D,
                    ld_qkv, ld_out);
  return mha_launch(qkv, ld_qkv, 0, xg, C, C, out, ld_out, n_images, P, H, D, stream);
}
