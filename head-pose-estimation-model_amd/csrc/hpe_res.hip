// hpe_res.hip — fused training of narrow residual stacks on gfx950: train_88.py's default graph,
// create_model_complex(reg, dr) (Model-88/attention_model.py:97-169, trained at train_88.py:309,
// 355-363: SGD, batch 128, 1x1 feature maps), and the stacks like it:
//
//   x (C_in = 88 | 96) -> dense 16 (act, SpatialDropout) -> NB x [dense 16 (act, drop) ->
//   dense 16 (act, drop) -> Add(block input) -> act] -> [dense BOT <= 16 (act, drop)] -> dense 3
//
// Every GEMM is an exact-fp32 v_mfma_f32_16x16x4_f32 over one 16-row block per wave (8 waves per
// workgroup), so the whole step is register-resident:
//   * "R-layout": lane (g, c) = (lane >> 4, lane & 15) holds row c of the block, features 4g .. 4g+3
//     of a 16-wide activation.  A forward layer computes Z^T = W^T . A^T: the weights are the A
//     operand (lane (g, c), K-step s: W[4g + s][c], read from the LDS copy of the parameters at each
//     use: conflict-free, and no registers held across layers), the R-layout input is the B operand
//     as it stands (K index 4g + s = its register s), and the output comes back in R-layout — no data
//     movement between layers.  The backward dA^T = W . dZ^T is the same with W[c][4g + s].
//   * dW = A^T . dZ sums over rows, so both operands must hold a feature per lane and rows over K
//     ("T-layout"): the wave transposes A and dZ through 2.5 KB of its own LDS (one ds_write_b128 and
//     four conflict-free ds_read_b32 each) and accumulates dW[in = 4g + i][out = c] in 4 registers
//     per 16x16 layer for the whole launch; the bias gradient is the same T-layout sum.
//   * the first layer's K = C_in runs as C_in / 4 K-steps with k = (C_in / 4) g + s: each lane reads
//     C_in / 4 contiguous floats of its row straight from HBM (the input never touches LDS); its dW
//     reads the input in T-layout (4 rows x 6 channel blocks per lane) from L2.
// The workgroup's 8 partial gradients are summed in a fixed tree order (deterministic) and either
// written to the workgroup's slab (hpe_train_step: hpe_reduce / hpe_reduce_optim_step follow) or,
// in the whole-epoch kernel, applied by the Keras legacy optimizer in the same launch
// (hpe_fit_epoch: parameters and Adam moments in LDS, one workgroup for the epoch).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/hpe.h"
#include "hpe_common.h"
#include "hpe_dev.h"

#define RES_NW 8                 // waves per workgroup: one 16-row block each
#define RES_T 16                 // rows per block
#define RES_SCR 640              // floats of a wave's transpose scratch: [2][16 rows][20]
#define RES_MAXP 4096            // trainable parameters held in LDS
#define RES_L_PRM 0
#define RES_L_M (RES_L_PRM + RES_MAXP)    // fit: optimizer moments
#define RES_L_V (RES_L_M + RES_MAXP)
#define RES_L_SCR (RES_L_V + RES_MAXP)
#define RES_L_RED (RES_L_SCR + RES_NW * RES_SCR)
#define RES_L_MISC (RES_L_RED + 4 * (RES_MAXP + 4))   // 4 flat partial-gradient copies
#define RES_LDS_FLOATS (RES_L_MISC + 64)
#define RES_LDS_BYTES (RES_LDS_FLOATS * 4)
static_assert(RES_LDS_BYTES <= 160 * 1024, "res LDS");

typedef float f4 __attribute__((ext_vector_type(4)));

// -DRES_STAMPS: per-phase s_memtime cycle sums of thread 0, printed at the end of the fit kernel
#ifdef RES_STAMPS
__device__ uint64_t g_rst[10];
__device__ uint64_t g_rprev;
#define RSTAMP(i) do { if (threadIdx.x == 0) { const uint64_t t_ = __builtin_amdgcn_s_memtime(); g_rst[i] += t_ - g_rprev; g_rprev = t_; } } while (0)
#else
#define RSTAMP(i) do {} while (0)
#endif

__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

template <int KS, int NB, bool BOTL>
struct ResGeo {
  static constexpr int CIN = 4 * KS;
  static constexpr int NL = 2 * NB + (BOTL ? 1 : 0) + 1;  // 16x16 layers after the first
  static constexpr int NLAY = NL + 1;
  static constexpr int NXB = (CIN + 15) / 16;             // 16-channel blocks of the first layer's dW
};

template <int KS, int NB, bool BOTL>
struct ResState {
  f4 acc0[ResGeo<KS, NB, BOTL>::NXB];     // dW0[16 b + 4g + i][c]
  f4 acc[ResGeo<KS, NB, BOTL>::NL];       // dW[4g + i][c]
  float dbp[ResGeo<KS, NB, BOTL>::NLAY];  // bias-gradient partial: feature c, rows 4g .. 4g+3
  float sse, sae;
};

// which rows a launch trains on: hpe_train_step rows (image = R / P, gathered by idx) or a
// whole-epoch step's batch (P = 1, rows perm[base + R])
struct RowMap {
  const int* idx;
  const int* perm;
  int64_t base, nrows, img_off;
  int P;
  bool fit;
  __device__ __forceinline__ int64_t label(int64_t R) const {
    if (fit) return perm[base + R];
    const int64_t im = R / P;
    return idx ? (int64_t)idx[im] : im;
  }
  __device__ __forceinline__ int64_t src(int64_t R) const {
    if (fit) return perm[base + R];
    const int64_t im = R / P;
    return (idx ? (int64_t)idx[im] : im) * P + (R - im * P);
  }
  __device__ __forceinline__ uint64_t dimg(int64_t R) const { return fit ? (uint64_t)R : (uint64_t)(R / P + img_off); }
};

// the layer activations on the hot path: softsign in a few VALU ops (reciprocal approximation,
// ~1 ulp relative), tanh as tanhf (these kernels are exact-fp32: hpe_dev.h fast_tanh5's absolute
// error bound is for the fp16-split kernels only), the rest as the interpreter computes them
__device__ __forceinline__ float res_act(int act, float z) {
  if (act == ACT_LINEAR) return z;
  if (act == ACT_SOFTSIGN) return z * __builtin_amdgcn_rcpf(1.f + fabsf(z));
  if (act == ACT_TANH) return tanhf(z);
  if (act == ACT_RELU) return z > 0.f ? z : 0.f;
  return act_f(act, z);
}
__device__ __forceinline__ float res_grad(int act, float a) {
  if (act == ACT_LINEAR) return 1.f;
  if (act == ACT_SOFTSIGN) {
    const float t = 1.f - fabsf(a);
    return t * t;
  }
  if (act == ACT_TANH) return 1.f - a * a;
  if (act == ACT_RELU) return a > 0.f ? 1.f : 0.f;
  return act_grad(act, a, 0.f);
}

// one dense layer: parameter offsets, K x N, activation, dropout (ordinal, threshold, 1 / keep)
struct LD {
  int wo, bo, K, N, act, drop;
  uint32_t thr;
  float ik;
};

// the layer table read ONCE per launch into registers (scalar loads of the program words inside the
// step loop are re-issued after every LDS / global store the compiler cannot disambiguate).  HA >= 0:
// the kernels compiled for create_model_complex's canonical geometry (first layer C_in x 16, blocks
// 16 x 16, bottleneck 16 x 8, output x 3, parameters packed in layer order, every hidden layer HA,
// the post-add activation relu, the output linear — checked on the host, res_fast): offsets, widths
// and activations are compile-time constants, only the dropout words are read
template <int KS, int NB, bool BOTL>
struct ResDesc {
  LD l[ResGeo<KS, NB, BOTL>::NLAY];
  int post;
};

template <int KS, int NB, bool BOTL>
__host__ __device__ constexpr int res_canon_k(int l) {
  return l == 0 ? 4 * KS : (l == ResGeo<KS, NB, BOTL>::NLAY - 1 ? (BOTL ? 8 : 16) : 16);
}
template <int KS, int NB, bool BOTL>
__host__ __device__ constexpr int res_canon_n(int l) {
  return l == ResGeo<KS, NB, BOTL>::NLAY - 1 ? 3 : ((BOTL && l == 2 * NB + 1) ? 8 : 16);
}
template <int KS, int NB, bool BOTL>
__host__ __device__ constexpr int res_canon_wo(int l) {
  int o = 0;
  for (int j = 0; j < l; ++j) o += res_canon_k<KS, NB, BOTL>(j) * res_canon_n<KS, NB, BOTL>(j) + res_canon_n<KS, NB, BOTL>(j);
  return o;
}

template <int KS, int NB, bool BOTL, int HA>
__device__ __forceinline__ ResDesc<KS, NB, BOTL> res_desc(const int* lt, int post) {
  using G = ResGeo<KS, NB, BOTL>;
  ResDesc<KS, NB, BOTL> D;
#pragma unroll
  for (int l = 0; l < G::NLAY; ++l) {
    const int* e = lt + l * RL_WORDS;
    LD& d = D.l[l];
    if (HA >= 0) {
      d.K = res_canon_k<KS, NB, BOTL>(l);
      d.N = res_canon_n<KS, NB, BOTL>(l);
      d.wo = res_canon_wo<KS, NB, BOTL>(l);
      d.bo = d.wo + d.K * d.N;
      d.act = l == G::NLAY - 1 ? ACT_LINEAR : HA;
    } else {
      d.K = e[RL_K];
      d.N = e[RL_N];
      d.wo = e[RL_W];
      d.bo = e[RL_B];
      d.act = e[RL_ACT];
    }
    d.drop = e[RL_DROP];
    d.thr = (uint32_t)e[RL_THR];
    d.ik = 1.f / __int_as_float(e[RL_KEEP]);
  }
  D.post = HA >= 0 ? ACT_RELU : post;
  return D;
}

// one dense layer's R-layout epilogue: a = act(z + b) (0 past N), kept bits, y = dropout(a)
// (nb0: the first feature of this 16-wide output block of a wider layer)
__device__ __forceinline__ f4 res_epi(f4 z, const float* prm, const LD& e, int g, uint64_t seed, uint64_t dimg,
                                      f4& a, uint32_t& km, int nb0 = 0) {
  const uint32_t base = e.drop >= 0 ? drop_base(seed, e.drop, dimg) : 0u;   // once per row and layer
  f4 y;
  km = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int n = nb0 + 4 * g + i;
    const float b = e.bo >= 0 ? prm[e.bo + min(n, e.N - 1)] : 0.f;
    const float v = n < e.N ? res_act(e.act, z[i] + b) : 0.f;
    a[i] = v;
    bool kp = true;
    if (e.drop >= 0) kp = drop_mix(base, (uint32_t)n) >= e.thr;
    km |= kp ? (1u << i) : 0u;
    y[i] = kp ? (e.drop >= 0 ? v * e.ik : v) : 0.f;
  }
  return y;
}

// y = dropout(a) again from the kept bits (the backward's layer input)
__device__ __forceinline__ f4 res_redrop(f4 a, const LD& e, uint32_t km) {
  f4 y;
#pragma unroll
  for (int i = 0; i < 4; ++i) y[i] = (km >> i) & 1u ? (e.drop >= 0 ? a[i] * e.ik : a[i]) : 0.f;
  return y;
}

// dL/dz of a layer from dL/dy through its dropout and activation (csrc/hpe_common.h epi_bwd)
__device__ __forceinline__ f4 res_epi_bwd(f4 dy, f4 a, const LD& e, uint32_t km) {
  f4 dz;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float gv = dy[i];
    if (e.drop >= 0) gv = (km >> i) & 1u ? gv * e.ik : 0.f;
    dz[i] = e.act == ACT_LINEAR ? gv : gv * res_grad(e.act, a[i]);
  }
  return dz;
}

// the weights are MFMA A operands read from the parameters in LDS at each use (all lanes of a
// 16-lane group read consecutive or broadcast words: conflict-free), not held in registers
// forward  Z^T = W^T . A^T: lane (g, c), K-step s: W[4g + s][c] (0 past K / N)
// (kb0 / nb0: the input / output block of a layer wider than 16; z: the accumulator to continue)
__device__ __forceinline__ f4 res_fwd16(const float* prm, const LD& e, int g, int c, f4 in, int kb0 = 0, int nb0 = 0,
                                        f4 z = f4{0.f, 0.f, 0.f, 0.f}) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int k = kb0 + 4 * g + s, n = nb0 + c;
    const float w = prm[e.wo + min(k, e.K - 1) * e.N + min(n, e.N - 1)];
    z = mfma4((k < e.K && n < e.N) ? w : 0.f, in[s], z);
  }
  return z;
}
// backward dA^T = W . dZ^T: lane (g, c), K-step s: W[c][4g + s]
__device__ __forceinline__ f4 res_bwd16(const float* prm, const LD& e, int g, int c, f4 dz, int kb0 = 0, int nb0 = 0) {
  f4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int n = nb0 + 4 * g + s, k = kb0 + c;
    const float w = prm[e.wo + min(k, e.K - 1) * e.N + min(n, e.N - 1)];
    d = mfma4((k < e.K && n < e.N) ? w : 0.f, dz[s], d);
  }
  return d;
}

// R-layout -> T-layout through the wave's scratch: out[s] = v[row 4g + s][feature c]
__device__ __forceinline__ void res_to_t(float* scr, f4 v, int g, int c, float (&out)[4]) {
  *(f4*)(scr + c * 20 + 4 * g) = v;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int s = 0; s < 4; ++s) out[s] = scr[(4 * g + s) * 20 + c];
}

// dW[in = 4g + i][out = c] += A^T . dZ over the block's 16 rows; bias partial += sum of dZ
__device__ __forceinline__ void res_dw16(f4& acc, float& dbp, f4 a_r, f4 dz_r, float* scr, int g, int c) {
  float at[4], dt[4];
  res_to_t(scr, a_r, g, c, at);
  res_to_t(scr + 320, dz_r, g, c, dt);
#pragma unroll
  for (int s = 0; s < 4; ++s) acc = mfma4(at[s], dt[s], acc);
  dbp += (dt[0] + dt[1]) + (dt[2] + dt[3]);
}

// forward + loss + backward of one 16-row block starting at batch row R0
template <int KS, int NB, bool BOTL>
__device__ __forceinline__ void res_block(ResState<KS, NB, BOTL>& S, const ResDesc<KS, NB, BOTL>& D,
                                          const float* prm, const float* __restrict__ x,
                                          const float* __restrict__ ytrue, const RowMap& rm, int64_t R0,
                                          uint64_t seed, float inv_count, float* scr, int g, int c) {
  using G = ResGeo<KS, NB, BOTL>;
  constexpr int CIN = G::CIN;
  const int64_t Rc = R0 + c;
  const bool valid = Rc < rm.nrows;
  const int64_t Rl = valid ? Rc : rm.nrows - 1;
  const uint64_t dimg = rm.dimg(Rl);
  const LD& e0 = D.l[0];
  const LD& eo = D.l[G::NLAY - 1];

  // ---- forward: first layer from HBM (row c, channels KS g .. KS g + KS - 1)
  f4 a0, y0;
  uint32_t m0;
  {
    const float* xp = x + rm.src(Rl) * CIN + KS * g;
    float xr[KS];
#pragma unroll
    for (int s = 0; s < KS; s += 2) {
      const float2 v = *(const float2*)(xp + s);
      xr[s] = v.x;
      xr[s + 1] = v.y;
    }
    const float* w0 = prm + e0.wo + KS * g * 16 + c;   // W0[KS g + s][c]
    f4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) z = mfma4(w0[16 * s], xr[s], z);
    y0 = res_epi(z, prm, e0, g, seed, dimg, a0, m0);
  }
  RSTAMP(0);
  // the first layer's dW reads the input in T-layout (rows 4g + s, channels 16 b + c): issued
  // now, consumed at the end of the backward
  float xt[G::NXB][4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int64_t R = min(R0 + 4 * g + s, rm.nrows - 1);
    const float* xp = x + rm.src(R) * CIN;
#pragma unroll
    for (int b = 0; b < G::NXB; ++b) {
      const int ch = 16 * b + c;
      const float v = xp[min(ch, CIN - 1)];
      xt[b][s] = ch < CIN ? v : 0.f;
    }
  }
  // ---- residual blocks
  f4 a1[NB], a2[NB], ho[NB];
  uint32_t m1[NB], m2[NB];
  f4 h = y0;
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const LD& e1 = D.l[2 * b + 1];
    const LD& e2 = D.l[2 * b + 2];
    const f4 y1 = res_epi(res_fwd16(prm, e1, g, c, h), prm, e1, g, seed, dimg, a1[b], m1[b]);
    const f4 y2 = res_epi(res_fwd16(prm, e2, g, c, y1), prm, e2, g, seed, dimg, a2[b], m2[b]);
#pragma unroll
    for (int i = 0; i < 4; ++i) ho[b][i] = res_act(D.post, h[i] + y2[i]);
    h = ho[b];
  }
  // ---- bottleneck, output
  f4 ab = {0.f, 0.f, 0.f, 0.f}, yb = h;
  uint32_t mb = 0;
  const LD& eb = D.l[BOTL ? 2 * NB + 1 : 0];
  if (BOTL) yb = res_epi(res_fwd16(prm, eb, g, c, h), prm, eb, g, seed, dimg, ab, mb);
  f4 ao;
  uint32_t mo;
  const f4 out = res_epi(res_fwd16(prm, eo, g, c, yb), prm, eo, g, seed, dimg, ao, mo);

  RSTAMP(1);
  // ---- MSE: lanes g = 0 hold the row's 3 outputs
  f4 dout = {0.f, 0.f, 0.f, 0.f};
  if (g == 0 && valid) {
    const float* yl = ytrue + rm.label(Rl) * 3;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const float err = out[i] - yl[i];
      S.sse = fmaf(err, err, S.sse);
      S.sae += fabsf(err);
      dout[i] = 2.f * err * inv_count;
    }
  }

  // ---- backward
  f4 dz = res_epi_bwd(dout, ao, eo, mo);
  res_dw16(S.acc[G::NL - 1], S.dbp[G::NLAY - 1], yb, dz, scr, g, c);
  f4 dh = res_bwd16(prm, eo, g, c, dz);
  if (BOTL) {
    dz = res_epi_bwd(dh, ab, eb, mb);
    res_dw16(S.acc[2 * NB], S.dbp[2 * NB + 1], h, dz, scr, g, c);
    dh = res_bwd16(prm, eb, g, c, dz);
  }
#pragma unroll
  for (int b = NB - 1; b >= 0; --b) {
    const LD& e1 = D.l[2 * b + 1];
    const LD& e2 = D.l[2 * b + 2];
    f4 ds;
#pragma unroll
    for (int i = 0; i < 4; ++i) ds[i] = D.post == ACT_LINEAR ? dh[i] : dh[i] * res_grad(D.post, ho[b][i]);
    const f4 dz2 = res_epi_bwd(ds, a2[b], e2, m2[b]);
    res_dw16(S.acc[2 * b + 1], S.dbp[2 * b + 2], res_redrop(a1[b], e1, m1[b]), dz2, scr, g, c);
    const f4 dz1 = res_epi_bwd(res_bwd16(prm, e2, g, c, dz2), a1[b], e1, m1[b]);
    const f4 hin = b == 0 ? y0 : ho[b > 0 ? b - 1 : 0];
    res_dw16(S.acc[2 * b], S.dbp[2 * b + 1], hin, dz1, scr, g, c);
    const f4 dx = res_bwd16(prm, e1, g, c, dz1);
    dh = ds + dx;
  }
  RSTAMP(2);
  // ---- first layer: dW0 += X^T . dZ0
  {
    const f4 dz0 = res_epi_bwd(dh, a0, e0, m0);
    float dt[4];
    res_to_t(scr + 320, dz0, g, c, dt);
#pragma unroll
    for (int b = 0; b < G::NXB; ++b)
#pragma unroll
      for (int s = 0; s < 4; ++s) S.acc0[b] = mfma4(xt[b][s], dt[s], S.acc0[b]);
    S.dbp[0] += (dt[0] + dt[1]) + (dt[2] + dt[3]);
  }
  RSTAMP(3);
}

template <int KS, int NB, bool BOTL>
__device__ __forceinline__ void res_zero(ResState<KS, NB, BOTL>& S) {
  using G = ResGeo<KS, NB, BOTL>;
#pragma unroll
  for (int b = 0; b < G::NXB; ++b) S.acc0[b] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int l = 0; l < G::NL; ++l) S.acc[l] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int l = 0; l < G::NLAY; ++l) S.dbp[l] = 0.f;
  S.sse = 0.f;
  S.sae = 0.f;
}

// a wave's partial gradient in the flat parameter layout: every trainable parameter of the stack
// is one dW / bias entry, so the wave writes (ADD = false) or adds onto (ADD = true) every word of
// out[0 .. npt) once, and out[npt], out[npt + 1] (sse, sae)
template <int KS, int NB, bool BOTL, bool ADD>
__device__ __forceinline__ void res_flat(const ResState<KS, NB, BOTL>& S, const ResDesc<KS, NB, BOTL>& D, float* out,
                                         int npt, int g, int c, int lane) {
  using G = ResGeo<KS, NB, BOTL>;
#define RES_PUT(idx, v) do { float* p_ = out + (idx); *p_ = ADD ? *p_ + (v) : (v); } while (0)
#pragma unroll
  for (int b = 0; b < G::NXB; ++b)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int in = 16 * b + 4 * g + i;
      if (in < G::CIN) RES_PUT(D.l[0].wo + in * 16 + c, S.acc0[b][i]);
    }
#pragma unroll
  for (int l = 0; l < G::NL; ++l) {
    const LD& e = D.l[l + 1];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int in = 4 * g + i;
      if (in < e.K && c < e.N) RES_PUT(e.wo + in * e.N + c, S.acc[l][i]);
    }
  }
#pragma unroll
  for (int l = 0; l < G::NLAY; ++l) {
    const LD& e = D.l[l];
    float v = S.dbp[l];
    v += __shfl_xor(v, 16, 64);
    v += __shfl_xor(v, 32, 64);
    if (g == 0 && e.bo >= 0 && c < e.N) RES_PUT(e.bo + c, v);
  }
  const float a = wave_sum(S.sse), b = wave_sum(S.sae);
  if (lane == 0) {
    RES_PUT(npt, a);
    RES_PUT(npt + 1, b);
  }
#undef RES_PUT
}

// the workgroup's 8 partial gradients: waves 4..7 write flat copies 0..3, waves 0..3 add theirs onto
// copy w, then every parameter i is ((c0 + c1) + (c2 + c3))[i] — a fixed order, identical in the
// per-step and whole-epoch kernels (bit-identical paths); returns after the barrier that publishes
template <int KS, int NB, bool BOTL>
__device__ __forceinline__ void res_reduce(const ResState<KS, NB, BOTL>& S, const ResDesc<KS, NB, BOTL>& D,
                                           float* cp, int npt, int stride, int wave, int g, int c, int lane) {
  if (wave >= 4) res_flat<KS, NB, BOTL, false>(S, D, cp + (wave - 4) * stride, npt, g, c, lane);
  __syncthreads();
  if (wave < 4) res_flat<KS, NB, BOTL, true>(S, D, cp + wave * stride, npt, g, c, lane);
  __syncthreads();
}

__device__ __forceinline__ float res_sum4(const float* cp, int stride, int i) {
  return (cp[i] + cp[stride + i]) + (cp[2 * stride + i] + cp[3 * stride + i]);
}

// The file is compiled five times (csrc/Makefile): RES_PART 88 / 96 with RES_FAST 0 / 1 instantiate
// the kernels of one input width and activation set, RES_PART 0 the host dispatch (the kernel
// instantiations take minutes to compile).
#ifndef RES_PART
#define RES_PART 0
#endif

// ---- hpe_train_step: per-workgroup gradient slabs ---------------------------------------------
template <int KS, int NB, bool BOTL, int HA>
__global__ void __launch_bounds__(RES_NW * 64) res_train_kernel(Args a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int* prog = a.prog;
  const int* o = prog + prog[H_OPS_OFF];
  const int* lt = prog + o[O_AUX0];
  const int npt = prog[H_NPARAMS_TRAIN];
  const int stride = (npt + 4 + 3) & ~3;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  float* prm = lds + RES_L_PRM;
  float* scr = lds + RES_L_SCR + wave * RES_SCR;
  float* cp = lds + RES_L_RED;
  for (int i = threadIdx.x; i < npt; i += RES_NW * 64) prm[i] = a.params[i];
  const ResDesc<KS, NB, BOTL> D = res_desc<KS, NB, BOTL, HA>(lt, o[O_MODE]);
  __syncthreads();
  ResState<KS, NB, BOTL> S;
  res_zero(S);
  RowMap rm = {a.idx, nullptr, 0, a.nrows, a.img_off, a.P, false};
  const int64_t nblk = (a.nrows + RES_T - 1) / RES_T;
  for (int64_t blk = (int64_t)blockIdx.x * RES_NW + wave; blk < nblk; blk += (int64_t)gridDim.x * RES_NW)
    res_block(S, D, prm, a.x, a.ytrue, rm, blk * RES_T, a.seed, a.inv_count, scr, g, c);
  res_reduce(S, D, cp, npt, stride, wave, g, c, lane);
  float* ws = a.ws + (size_t)blockIdx.x * prog[H_SLAB];
  for (int i = threadIdx.x; i < npt + 2; i += RES_NW * 64) ws[i] = res_sum4(cp, stride, i);
  if (threadIdx.x < 2) ws[npt + 2 + threadIdx.x] = 0.f;
}

// ---- hpe_fit_epoch: the whole epoch in one workgroup ------------------------------------------------
struct ResFitArgs {
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
  const float* alpha;       // [steps] step sizes (lr for SGD), host-computed as hpe_optim_step
  uint64_t seed_base;       // dropout seed of step s = seed_base + iter0 + 1 + s
  int64_t iter0;
  float* stats;             // [steps][stats_stride]: sse, sae, regularisation loss
  int stats_stride;
  int* flags;               // workspace word 1 (always 0: exact fp32 throughout)
};

// one step of the Keras legacy optimizer over the workgroup's parameters in LDS from the summed
// flat gradient copies (hpe_rowprog.hip optim_update with gscale 1: the same float operations), the
// regularisation loss on the pre-update weights, and the step's stats row
__device__ __forceinline__ float res_opt_one(const ResFitArgs& a, float alpha, float wi, float c2, float g,
                                             float& mi, float& vi) {
  const float gr = fmaf(g, 1.f, 2.f * c2 * wi);
  if (a.kind == HPE_OPT_SGD) return wi - alpha * gr;
  if (a.kind == HPE_OPT_ADAM) {
    mi += (gr - mi) * (1.f - a.b1);
    vi += (gr * gr - vi) * (1.f - a.b2);
    return wi - (mi * alpha) / (sqrtf(vi) + a.eps);
  }
  mi += (gr - mi) * (1.f - a.b1);
  vi = fmaxf(a.b2 * vi, fabsf(gr));
  return wi - alpha * (mi / (vi + a.eps));
}

__device__ __forceinline__ void res_opt_step(const ResFitArgs& a, float* prm, float* mom, float* vel, const float* cp,
                                             int stride, int npt, int s, float* misc, int tid, int lane, int wave) {
  const float alpha = a.alpha[s];
  float reg = 0.f;
  for (int i = tid; i < npt; i += RES_NW * 64) {
    const float wi = prm[i], c2 = a.l2[i];
    reg = fmaf(c2 * wi, wi, reg);
    float mi = mom[i], vi = vel[i];
    prm[i] = res_opt_one(a, alpha, wi, c2, res_sum4(cp, stride, i), mi, vi);
    if (a.kind != HPE_OPT_SGD) {
      mom[i] = mi;
      vel[i] = vi;
    }
  }
  reg = wave_sum(reg);
  if (lane == 0) misc[wave] = reg;
  // the copies are read before the barrier (the next step's reduction overwrites them after it)
  const float sse = res_sum4(cp, stride, npt), sae = res_sum4(cp, stride, npt + 1);
  __syncthreads();
  if (tid == 0) {
    float* st = a.stats + (size_t)s * a.stats_stride;
    st[0] = sse;
    st[1] = sae;
    st[2] = ((misc[0] + misc[1]) + (misc[2] + misc[3])) + ((misc[4] + misc[5]) + (misc[6] + misc[7]));
  }
}

template <int KS, int NB, bool BOTL, int HA>
__global__ void __launch_bounds__(RES_NW * 64) res_fit_kernel(ResFitArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int* prog = a.prog;
  const int* o = prog + prog[H_OPS_OFF];
  const int* lt = prog + o[O_AUX0];
  const int npt = prog[H_NPARAMS_TRAIN];
  const int stride = (npt + 4 + 3) & ~3;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, g = lane >> 4, c = lane & 15;
  const int tid = threadIdx.x;
  float* prm = lds + RES_L_PRM;
  float* mom = lds + RES_L_M;
  float* vel = lds + RES_L_V;
  float* scr = lds + RES_L_SCR + wave * RES_SCR;
  float* cp = lds + RES_L_RED;
  float* misc = lds + RES_L_MISC;
  for (int i = tid; i < npt; i += RES_NW * 64) {
    prm[i] = a.params[i];
    mom[i] = a.kind != HPE_OPT_SGD ? a.m[i] : 0.f;
    vel[i] = a.kind != HPE_OPT_SGD ? a.v[i] : 0.f;
  }
  if (tid == 0) a.flags[1] = 0;
  const ResDesc<KS, NB, BOTL> D = res_desc<KS, NB, BOTL, HA>(lt, o[O_MODE]);
  __syncthreads();
  ResState<KS, NB, BOTL> S;
#ifdef RES_STAMPS
  if (threadIdx.x == 0) {
    for (int i = 0; i < 10; ++i) g_rst[i] = 0;
    g_rprev = __builtin_amdgcn_s_memtime();
  }
#endif
  for (int s = 0; s < a.steps; ++s) {
    const int64_t base = (int64_t)s * a.bs;
    const int nb = (int)min((int64_t)a.bs, (int64_t)a.n - base);
    res_zero(S);
    RowMap rm = {nullptr, a.perm, base, nb, 0, 1, true};
    const uint64_t seed = a.seed_base + (uint64_t)(a.iter0 + 1 + s);
    const float inv = 1.f / (float)(nb * 3);
    const int nblk = (nb + RES_T - 1) / RES_T;
    for (int blk = wave; blk < nblk; blk += RES_NW)
      res_block(S, D, prm, a.x, a.ytrue, rm, (int64_t)blk * RES_T, seed, inv, scr, g, c);
    res_reduce(S, D, cp, npt, stride, wave, g, c, lane);
    RSTAMP(4);
    res_opt_step(a, prm, mom, vel, cp, stride, npt, s, misc, tid, lane, wave);
    RSTAMP(5);
  }
#ifdef RES_STAMPS
  if (threadIdx.x == 0)
    printf("RSTAMP steps %d: fwd0 %llu fwd %llu bwd %llu dw0 %llu reduce %llu opt %llu\n", a.steps,
           (unsigned long long)g_rst[0], (unsigned long long)g_rst[1], (unsigned long long)g_rst[2],
           (unsigned long long)g_rst[3], (unsigned long long)g_rst[4], (unsigned long long)g_rst[5]);
#endif
  for (int i = tid; i < npt; i += RES_NW * 64) {
    const float w = prm[i];
    a.params[i] = w;
    const int tp = a.tpos[i];
    if (tp >= 0) a.params_t[tp] = w;
    if (a.kind != HPE_OPT_SGD) {
      a.m[i] = mom[i];
      a.v[i] = vel[i];
    }
  }
}

// ---- host side ----------------------------------------------------------------------------------
typedef void (*res_train_fn)(Args);
typedef void (*res_fit_fn)(ResFitArgs);

#ifndef RES_FAST
#define RES_FAST 0
#endif
#define RES_HA (RES_FAST ? ACT_SOFTSIGN : -1)
#if RES_PART != 0
template <int KS, bool BOTL>
static void res_pick_nb(int nb, res_train_fn* t, res_fit_fn* f) {
  switch (nb) {
    case 1: *t = res_train_kernel<KS, 1, BOTL, RES_HA>; *f = res_fit_kernel<KS, 1, BOTL, RES_HA>; break;
    case 2: *t = res_train_kernel<KS, 2, BOTL, RES_HA>; *f = res_fit_kernel<KS, 2, BOTL, RES_HA>; break;
    case 3: *t = res_train_kernel<KS, 3, BOTL, RES_HA>; *f = res_fit_kernel<KS, 3, BOTL, RES_HA>; break;
    case 4: *t = res_train_kernel<KS, 4, BOTL, RES_HA>; *f = res_fit_kernel<KS, 4, BOTL, RES_HA>; break;
    default: break;
  }
}
#define RES_FNS_NAME3(n, f) res_fns_##n##_##f
#define RES_FNS_NAME(n, f) RES_FNS_NAME3(n, f)
// a residual stack of nb blocks (bot: with the bottleneck)
void RES_FNS_NAME(RES_PART, RES_FAST)(int nb, bool bot, res_train_fn* t, res_fit_fn* f) {
  if (bot) res_pick_nb<RES_PART / 4, true>(nb, t, f);
  else res_pick_nb<RES_PART / 4, false>(nb, t, f);
}
#else
void res_fns_88_0(int nb, bool bot, res_train_fn* t, res_fit_fn* f);
void res_fns_88_1(int nb, bool bot, res_train_fn* t, res_fit_fn* f);
void res_fns_96_0(int nb, bool bot, res_train_fn* t, res_fit_fn* f);
void res_fns_96_1(int nb, bool bot, res_train_fn* t, res_fit_fn* f);

// the compile-time-activation kernels: every hidden dense softsign, the post-add activation relu,
// the output linear (create_model_complex, Model-88/attention_model.py:97-169)
static bool res_fast(const int* w) {
  const int* o = w + w[H_OPS_OFF];
  const int* lt = w + o[O_AUX0];
  const int L = o[O_AUX1], cin = o[O_K], nb = o[O_AUX3], bot = o[O_FLAGS];
  if (o[O_MODE] != ACT_RELU || (bot != 0 && bot != 8)) return false;
  int off = 0;
  for (int l = 0; l < L; ++l) {
    const int* e = lt + l * RL_WORDS;
    const int K = l == 0 ? cin : (l == L - 1 ? (bot ? 8 : 16) : 16);
    const int N = l == L - 1 ? 3 : ((bot && l == 2 * nb + 1) ? 8 : 16);
    if (e[RL_K] != K || e[RL_N] != N || e[RL_W] != off || e[RL_B] != off + K * N) return false;
    if (e[RL_ACT] != (l == L - 1 ? ACT_LINEAR : ACT_SOFTSIGN)) return false;
    off += K * N + N;
  }
  return off == w[H_NPARAMS_TRAIN];
}

static bool res_pick(const int* w, res_train_fn* t, res_fit_fn* f) {
  *t = nullptr;
  *f = nullptr;
  const int* o = w + w[H_OPS_OFF];
  if (o[O_TYPE] != OP_RES) return false;
  const int cin = o[O_K], nb = o[O_AUX3], F = o[O_N];
  const bool bot = o[O_FLAGS] > 0;
  if (nb <= 0 || F != 16 || o[O_AUX1] != 2 * nb + 2 + (bot ? 1 : 0)) return false;
  const bool fast = res_fast(w);
  if (cin == 88) (fast ? res_fns_88_1 : res_fns_88_0)(nb, bot, t, f);
  else if (cin == 96) (fast ? res_fns_96_1 : res_fns_96_0)(nb, bot, t, f);
  return *t != nullptr;
}
int res_supported(const int* w) {
  res_train_fn t;
  res_fit_fn f;
  return w[H_MODE] == MODE_TRAIN && w[H_NPARAMS_TRAIN] <= RES_MAXP && res_pick(w, &t, &f) ? 1 : 0;
}

int res_grid_cap(int n_cu) { return n_cu; }

int res_launch(const int* w, const Args& a, int grid, hipStream_t s) {
  res_train_fn t;
  res_fit_fn f;
  if (!res_pick(w, &t, &f)) return 2;
  const int lds = RES_LDS_BYTES;
  hipFuncSetAttribute((const void*)t, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  const int tv = hpe_tev_begin(s);
  hipLaunchKernelGGL(t, dim3(grid), dim3(RES_NW * 64), lds, s, a);
  hpe_tev_end(s, tv);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

int res_fit_launch(const int* w, const int* dwords, float* params, float* params_t, float* m, float* v,
                   const float* l2, const int32_t* tpos, const float* x, const float* y_true, const int32_t* perm,
                   int64_t n, int32_t batch, int32_t kind, float beta_1, float beta_2, float epsilon,
                   const float* alpha, uint64_t seed_base, int64_t iter0, float* stats, int32_t stats_stride,
                   void* workspace, hipStream_t s) {
  res_train_fn t;
  res_fit_fn f;
  if (!res_pick(w, &t, &f)) return 2;
  ResFitArgs a = {};
  a.prog = dwords;
  a.params = params; a.params_t = params_t; a.m = m; a.v = v; a.l2 = l2; a.tpos = tpos;
  a.x = x; a.ytrue = y_true; a.perm = perm;
  a.n = (int)n; a.bs = batch; a.steps = (int)((n + batch - 1) / batch); a.kind = kind;
  a.b1 = beta_1; a.b2 = beta_2; a.eps = epsilon;
  a.alpha = alpha; a.seed_base = seed_base; a.iter0 = iter0;
  a.stats = stats; a.stats_stride = stats_stride;
  a.flags = (int*)workspace;
  const int lds = RES_LDS_BYTES;
  hipFuncSetAttribute((const void*)f, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  const int tv = hpe_tev_begin(s);
  hipLaunchKernelGGL(f, dim3(1), dim3(RES_NW * 64), lds, s, a);
  hpe_tev_end(s, tv);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
#endif
