// hpe_tail.hip — the row-local tail of the reference's SE-Transformer attention head on H x W > 1
// maps (Model-88/attention_model.py:56-72, se_transformer_regr_head) in ONE kernel, after the
// attention core (hpe_mha_xg):
//
//   t = xg + o . Wo + bo            residual Add(flat, MultiHeadAttention output)   :56
//   u = LayerNorm(t)                                                                  :57
//   v = act(u . Wf1 + bf1)          feed-forward Dense(ff_dim, relu)                  :60
//   w = u + (v . Wf2 + bf2)         Dense(C), residual Add                            :61-62
//   z = LayerNorm(w)                                                                  :63
//   h = act(z . Wc1 + bc1)          Conv2D(hidden, 1x1, relu)                         :70
//   y = h . Wc2 + bc2               Conv2D(3, 1x1)                                     :71
//
// Every row is independent: one wave runs a 16-row block through the whole chain in registers
// ("R-layout": lane (g, c) = (lane >> 4, lane & 15) holds row c, features 16 b + 4 g .. +3 of block b),
// each GEMM as Z^T = W^T . A^T on exact-fp32 v_mfma_f32_16x16x4_f32 with the layer input as the B
// operand exactly as the previous layer left it.  The weights live in LDS, pre-arranged on the host
// in MFMA operand order (one ds_read_b128 feeds four MFMAs, conflict-free); the residual Add of the
// attention output is an add of xg in the epilogue, not an [I; Wo] GEMM; LayerNorm's row sums are an
// in-lane sum plus two cross-lane steps.  HBM traffic per row: xg (C floats), o (H D floats), 3 out.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hpe.h"
#include "hpe_common.h"

#define TL_NW 8                  // waves per workgroup (one 16-row block each)

typedef float f4 __attribute__((ext_vector_type(4)));

// host descriptor words (hpe/spatial.py AttnTail.desc)
enum {
  TD_C = 0, TD_HD, TD_FF, TD_HID, TD_ACT_FF, TD_ACT_HID, TD_ACT_OUT, TD_EPS1, TD_EPS2, TD_NW,
  TD_BO, TD_G1, TD_BE1, TD_BF1, TD_BF2, TD_G2, TD_BE2, TD_BC1, TD_BC2, TD_WORDS = 20
};

struct TailArgs {
  const float* xg;
  const float* o;
  float* y;
  const float* w;   // prepared parameters (weights in MFMA order, then the vectors)
  int64_t nrows;
  int ld_xg, ld_o;
  int d[TD_WORDS];
};

__device__ __forceinline__ f4 mfma4t(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// z[bn] = sum_k x[k] W[k][16 bn + c] for all NB output blocks; W pre-arranged as
// [KB][NB][g][c][s] = W[16 bk + 4g + s][16 bn + c] (zero padded)
template <int KB, int NB>
__device__ __forceinline__ void tl_dense(const float* wl, const f4 (&x)[KB], f4 (&z)[NB], int lane) {
#pragma unroll
  for (int bn = 0; bn < NB; ++bn) z[bn] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int bk = 0; bk < KB; ++bk) {
#pragma unroll
    for (int bn = 0; bn < NB; ++bn) {
      const f4 wv = *(const f4*)(wl + ((bk * NB + bn) * 64 + lane) * 4);
#pragma unroll
      for (int s = 0; s < 4; ++s) z[bn] = mfma4t(wv[s], x[bk][s], z[bn]);
    }
    // one K block's weights in flight at a time (hoisting them all spills)
    __builtin_amdgcn_sched_barrier(0);
  }
}

__device__ __forceinline__ float tl_act(int act, float z) {
  if (act == ACT_LINEAR) return z;
  if (act == ACT_RELU) return z > 0.f ? z : 0.f;
  return act_f(act, z);
}

template <int NB>
__device__ __forceinline__ void tl_bias_act(f4 (&z)[NB], const float* b, int act, int g) {
#pragma unroll
  for (int bn = 0; bn < NB; ++bn) {
    const f4 bv = *(const f4*)(b + 16 * bn + 4 * g);
#pragma unroll
    for (int i = 0; i < 4; ++i) z[bn][i] = tl_act(act, z[bn][i] + bv[i]);
  }
}

// LayerNorm over the first C features of each row (features past C are zero and stay zero:
// gamma / beta are zero padded)
template <int NB>
__device__ __forceinline__ void tl_layernorm(f4 (&x)[NB], const float* gamma, const float* beta, float eps, int C,
                                             int g) {
  float s = 0.f;
#pragma unroll
  for (int b = 0; b < NB; ++b) s += (x[b][0] + x[b][1]) + (x[b][2] + x[b][3]);
  s += __shfl_xor(s, 16, 64);
  s += __shfl_xor(s, 32, 64);
  const float mu = s / (float)C;
  float q = 0.f;
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float d = 16 * b + 4 * g + i < C ? x[b][i] - mu : 0.f;
      q = fmaf(d, d, q);
    }
  q += __shfl_xor(q, 16, 64);
  q += __shfl_xor(q, 32, 64);
  const float rstd = 1.f / sqrtf(q / (float)C + eps);
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const f4 gv = *(const f4*)(gamma + 16 * b + 4 * g), bv = *(const f4*)(beta + 16 * b + 4 * g);
#pragma unroll
    for (int i = 0; i < 4; ++i) x[b][i] = fmaf((x[b][i] - mu) * rstd, gv[i], bv[i]);
  }
}

template <int CB, int HB, int FB, int NHB>
__global__ void __launch_bounds__(TL_NW * 64) attn_tail_kernel(TailArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  const int nw = a.d[TD_NW];
  {
    const f4* src = (const f4*)a.w;
    f4* dst = (f4*)lds;
    for (int i = threadIdx.x; i < nw / 4; i += TL_NW * 64) dst[i] = src[i];
  }
  __syncthreads();
  const float* w_o = lds;                               // [HB][CB] blocks
  const float* w_f1 = w_o + HB * CB * 256;              // [CB][FB]
  const float* w_f2 = w_f1 + CB * FB * 256;             // [FB][CB]
  const float* w_c1 = w_f2 + FB * CB * 256;             // [CB][NHB]
  const float* w_c2 = w_c1 + CB * NHB * 256;            // [NHB][1]
  const int C = a.d[TD_C], HD = a.d[TD_HD];
  const int act_ff = a.d[TD_ACT_FF], act_hid = a.d[TD_ACT_HID], act_out = a.d[TD_ACT_OUT];
  const float eps1 = __int_as_float(a.d[TD_EPS1]), eps2 = __int_as_float(a.d[TD_EPS2]);
  const int64_t nblk = (a.nrows + 15) / 16;
  for (int64_t blk = (int64_t)blockIdx.x * TL_NW + wave; blk < nblk; blk += (int64_t)gridDim.x * TL_NW) {
    const int64_t row = blk * 16 + c;
    const int64_t rl = row < a.nrows ? row : a.nrows - 1;
    f4 xo[HB], t[CB];
    {
      const float* op = a.o + rl * a.ld_o + 4 * g;
#pragma unroll
      for (int b = 0; b < HB; ++b) xo[b] = 16 * b + 4 * g < HD ? *(const f4*)(op + 16 * b) : f4{0.f, 0.f, 0.f, 0.f};
    }
    tl_dense<HB, CB>(w_o, xo, t, lane);
    {
      const float* xp = a.xg + rl * a.ld_xg + 4 * g;
      const float* bo = lds + a.d[TD_BO];
#pragma unroll
      for (int b = 0; b < CB; ++b) {
        const f4 xv = 16 * b + 4 * g < C ? *(const f4*)(xp + 16 * b) : f4{0.f, 0.f, 0.f, 0.f};
        const f4 bv = *(const f4*)(bo + 16 * b + 4 * g);
        t[b] = (t[b] + bv) + xv;
      }
    }
    tl_layernorm<CB>(t, lds + a.d[TD_G1], lds + a.d[TD_BE1], eps1, C, g);
    f4 v[FB];
    tl_dense<CB, FB>(w_f1, t, v, lane);
    tl_bias_act<FB>(v, lds + a.d[TD_BF1], act_ff, g);
    f4 u[CB];
    tl_dense<FB, CB>(w_f2, v, u, lane);
    {
      const float* bf2 = lds + a.d[TD_BF2];
#pragma unroll
      for (int b = 0; b < CB; ++b) u[b] = t[b] + (u[b] + *(const f4*)(bf2 + 16 * b + 4 * g));
    }
    tl_layernorm<CB>(u, lds + a.d[TD_G2], lds + a.d[TD_BE2], eps2, C, g);
    f4 h[NHB];
    tl_dense<CB, NHB>(w_c1, u, h, lane);
    tl_bias_act<NHB>(h, lds + a.d[TD_BC1], act_hid, g);
    f4 out[1];
    tl_dense<NHB, 1>(w_c2, h, out, lane);
    if (g == 0 && row < a.nrows) {
      const float* bc2 = lds + a.d[TD_BC2];
#pragma unroll
      for (int i = 0; i < 3; ++i) a.y[row * 3 + i] = tl_act(act_out, out[0][i] + bc2[i]);
    }
  }
}

typedef void (*tail_fn)(TailArgs);

template <int CB, int HB>
static tail_fn tail_pick2(int fb, int nhb) {
  if (fb == 4 && nhb == 8) return attn_tail_kernel<CB, HB, 4, 8>;
  if (fb == 4 && nhb == 4) return attn_tail_kernel<CB, HB, 4, 4>;
  if (fb == 2 && nhb == 8) return attn_tail_kernel<CB, HB, 2, 8>;
  return nullptr;
}

static tail_fn tail_pick(int cb, int hb, int fb, int nhb) {
  if (cb == 6 && hb == 4) return tail_pick2<6, 4>(fb, nhb);   // C 88 (se_transformer_regr_head), 4 x 16
  if (cb == 6 && hb == 2) return tail_pick2<6, 2>(fb, nhb);   // 4 heads x key_dim 8
  if (cb == 6 && hb == 1) return tail_pick2<6, 1>(fb, nhb);   // 4 heads x key_dim <= 4
  if (cb == 6 && hb == 8) return tail_pick2<6, 8>(fb, nhb);
  return nullptr;
}

static int tail_blocks(int n) { return (n + 15) / 16; }

extern "C" int hpe_attn_tail_supported(const int32_t* d) {
  if (!d) return 0;
  if (d[TD_C] < 4 || d[TD_C] % 4 || d[TD_HD] < 4 || d[TD_HD] % 4) return 0;
  const int cb = tail_blocks(d[TD_C]), hb = tail_blocks(d[TD_HD]), fb = tail_blocks(d[TD_FF]), nhb = tail_blocks(d[TD_HID]);
  if (!tail_pick(cb, hb, fb, nhb)) return 0;
  return d[TD_NW] > 0 && (int64_t)d[TD_NW] * 4 <= 160 * 1024 && d[TD_NW] % 4 == 0;
}

extern "C" int hpe_attn_tail(const float* xg, int32_t ld_xg, const float* o, int32_t ld_o, int64_t n_rows,
                             const int32_t* desc, const float* w, float* y, void* stream) {
  if (!xg || !o || !desc || !w || !y) return hpe_fail(HPE_EINVAL, "hpe_attn_tail: null argument");
  if (!hpe_attn_tail_supported(desc)) return hpe_fail(HPE_EINVAL, "hpe_attn_tail: unsupported geometry");
  if (n_rows <= 0) return 0;
  if (ld_xg < desc[TD_C] || ld_o < desc[TD_HD] || ld_xg % 4 || ld_o % 4)
    return hpe_fail(HPE_EINVAL, "hpe_attn_tail: bad strides %d %d", ld_xg, ld_o);
  TailArgs a = {};
  a.xg = xg; a.o = o; a.y = y; a.w = w; a.nrows = n_rows; a.ld_xg = ld_xg; a.ld_o = ld_o;
  for (int i = 0; i < TD_WORDS; ++i) a.d[i] = desc[i];
  const tail_fn k = tail_pick(tail_blocks(desc[TD_C]), tail_blocks(desc[TD_HD]), tail_blocks(desc[TD_FF]),
                              tail_blocks(desc[TD_HID]));
  const int lds = desc[TD_NW] * 4;
  int dev = 0, ncu = 256;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const int64_t blocks = (n_rows + 16 * TL_NW - 1) / (16 * TL_NW);
  const int grid = (int)(blocks < ncu ? blocks : ncu);
  hipStream_t s = (hipStream_t)stream;
  if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess)
    return hpe_fail(HPE_ERUNTIME, "hpe_attn_tail: LDS attribute");
  const int tv = hpe_tev_begin(s);
  hipLaunchKernelGGL(k, dim3(grid), dim3(TL_NW * 64), lds, s, a);
  hpe_tev_end(s, tv);
  return hipGetLastError() == hipSuccess ? 0 : hpe_fail(HPE_ERUNTIME, "hpe_attn_tail: launch failed");
}
