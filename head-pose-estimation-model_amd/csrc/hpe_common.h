// hpe_common.h — device helpers shared by the row-program interpreter and the fused kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "hpe_prog.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define MAXTHIN 4

// ------------------------------------------------------------------------------------------------
// activations and their derivatives (derivative from the stored output where possible)
// ------------------------------------------------------------------------------------------------
#define SELU_ALPHA 1.6732632423543772848170429916717f
#define SELU_SCALE 1.0507009873554804934193349852946f

__device__ __forceinline__ float act_f(int act, float z) {
  switch (act) {
    case ACT_TANH: return tanhf(z);
    case ACT_RELU: return z > 0.f ? z : 0.f;
    case ACT_SOFTSIGN: return z / (1.f + fabsf(z));
    case ACT_SIGMOID: return 1.f / (1.f + expf(-z));
    case ACT_ELU: return z > 0.f ? z : expm1f(z);
    case ACT_SELU: return SELU_SCALE * (z > 0.f ? z : SELU_ALPHA * expm1f(z));
    case ACT_SWISH: return z / (1.f + expf(-z));
    case ACT_SOFTPLUS: return z > 20.f ? z : log1pf(expf(z));
    case ACT_LEAKY_RELU: return z > 0.f ? z : 0.2f * z;
    default: return z;
  }
}

// d act / dz given a = act(z) (and z for swish)
__device__ __forceinline__ float act_grad(int act, float a, float z) {
  switch (act) {
    case ACT_TANH: return 1.f - a * a;
    case ACT_RELU: return a > 0.f ? 1.f : 0.f;
    case ACT_SOFTSIGN: { float t = 1.f - fabsf(a); return t * t; }
    case ACT_SIGMOID: return a * (1.f - a);
    case ACT_ELU: return a > 0.f ? 1.f : a + 1.f;
    case ACT_SELU: return a > 0.f ? SELU_SCALE : a + SELU_SCALE * SELU_ALPHA;
    case ACT_SWISH: { float s = 1.f / (1.f + expf(-z)); return s * (1.f + z * (1.f - s)); }
    case ACT_SOFTPLUS: return -expm1f(-a);
    case ACT_LEAKY_RELU: return a > 0.f ? 1.f : 0.2f;
    default: return 1.f;
  }
}

// SpatialDropout2D keep test: counter hash of (seed, dropout ordinal, image, channel), restated
// bit-for-bit by oracle/keras_ref.py:dropout_hash.  One 64-bit splitmix of (seed, ordinal, image) —
// the same for every channel of an image, so a kernel computing several channels of one image pays
// it once (the compiler shares it) — then a 32-bit murmur3 finaliser of (base, channel) per channel.
__device__ __forceinline__ uint32_t drop_base(uint64_t seed, int drop_id, uint64_t image) {
  uint64_t x = seed + 0x9E3779B97F4A7C15ull * (uint64_t)(1 + drop_id);
  x ^= image * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  x ^= x >> 31;
  return (uint32_t)(x >> 32);
}
__device__ __forceinline__ uint32_t drop_mix(uint32_t base, uint32_t c) {
  uint32_t h = base ^ (c * 0x9E3779B9u);
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}
__device__ __forceinline__ uint32_t drop_hash(uint64_t seed, int drop_id, uint64_t image, uint32_t c) {
  return drop_mix(drop_base(seed, drop_id, image), c);
}

struct Epi {
  int act, drop, zslot;
  uint32_t thr;
  float keep;
};

// program words read through the constant address space: the words never change during a launch,
// so uniform reads become scalar loads instead of vector loads that the compiler must re-issue
// (behind a vmcnt(0)) after every store it cannot prove disjoint from the program
typedef const __attribute__((address_space(4))) int pword;

struct Ctx {
  const pword* prog;
  const float* params;
  const float* params_t;
  float* lds;
  int T;
  int64_t row0;     // first row of the tile (batch-local)
  int64_t nrows;    // valid rows
  int P;            // positions per image
  int64_t img_off;  // global index of this launch's first image (dropout hash)
  uint64_t seed;
};

__device__ __forceinline__ int slot_w(const Ctx& c, int s, int w) {
  return c.prog[c.prog[H_SLOTS_OFF] + s * S_WORDS + w];
}

template <typename W>
__device__ __forceinline__ Epi load_epi(const W* o) {
  Epi e;
  e.act = o[O_EACT];
  e.drop = o[O_EDROP];
  e.zslot = o[O_EZ];
  e.thr = (uint32_t)o[O_ETHR];
  e.keep = __int_as_float(o[O_EKEEP]);
  return e;
}

__device__ __forceinline__ int64_t image_of(const Ctx& c, int r) {
  return (c.row0 + r) / c.P + c.img_off;
}

__device__ __forceinline__ float epi_fwd(const Ctx& c, const Epi& e, float z, int r, int ch) {
  float a = act_f(e.act, z);
  if (e.drop >= 0) a = drop_hash(c.seed, e.drop, image_of(c, r), ch) >= e.thr ? a / e.keep : 0.f;
  return a;
}

// gradient through the epilogue: g = dL/d(stored output), val = stored output
__device__ __forceinline__ float epi_bwd(const Ctx& c, const Epi& e, float g, float val, float z,
                                         int r, int ch) {
  if (e.drop >= 0) {
    if (drop_hash(c.seed, e.drop, image_of(c, r), ch) < e.thr) return 0.f;
    g = g / e.keep;
    val = val * e.keep;
  }
  return e.act == ACT_LINEAR ? g : g * act_grad(e.act, val, z);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// lane l <-> lane l ^ 32 in one VALU op (gfx950 v_permlane32_swap) instead of an LDS-pipe bpermute
__device__ __forceinline__ float xor32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float((__lane_id() & 32) ? r[0] : r[1]);
}

// wave-wide sum on DPP (VALU: quad_perm, row mirrors, row broadcasts) in a fixed order, the total
// broadcast from lane 63; a __shfl_xor butterfly is six dependent LDS-pipe round trips instead
#define DPP_SUM_STEP(v, ctrl, rmask) v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), ctrl, rmask, 0xf, false))
__device__ __forceinline__ float wave_sum_dpp(float v) {
  DPP_SUM_STEP(v, 0xB1, 0xf);   // quad_perm [1,0,3,2]
  DPP_SUM_STEP(v, 0x4E, 0xf);   // quad_perm [2,3,0,1]
  DPP_SUM_STEP(v, 0x141, 0xf);  // row_half_mirror
  DPP_SUM_STEP(v, 0x140, 0xf);  // row_mirror: every lane holds its row's sum
  DPP_SUM_STEP(v, 0x142, 0xa);  // row_bcast:15 -> rows 1, 3
  DPP_SUM_STEP(v, 0x143, 0xc);  // row_bcast:31 -> rows 2, 3: lane 63 holds the total
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// guarded (fp16-split) launches: a ring of guard words per program, indexed by launch epoch; the
// word HPE_GUARD_RING past a launch's guard word collects which check fired (diagnostics)
#define HPE_GUARD_RING 16

struct Args {
  const int* prog;
  const float* params;
  const float* params_t;
  const float* x;
  const float* ytrue;
  const int* idx;
  float* y;          // forward output
  float* ws;         // per-workgroup partials (train / eval)
  int64_t nrows;
  int P;
  int64_t img_off;
  float inv_count;
  uint64_t seed;
  int* guard;        // fp16-split kernels: set to `epoch` when a tile's split overflowed (non-finite)
  int epoch;         //   -> the exact-fp32 kernel of the same launch re-runs (guard == epoch)
  float* gscr;       // rowprog_kernel<..., GS = true>: per-workgroup slot scratch (H_GSLOTS programs)
  int pass;          // rowprog_kernel: dW-block pass of a multi-pass (H_NPASS) training program
  const float* wsplit;  // rowprog_kernel<..., SPLIT = true>: pre-split OP_DENSE weights (O_AUX3 offsets)
  float x_bound;        // caller's bound on max |x| (0: unknown); < the split's data range: no exact twin
};

// the fp16 split's data-side range (|d| < 65504 / 2^SPLIT_SHIFT): a launch whose inputs are known to
// lie below it cannot overflow on the data side (the weight / dZ sides are power-of-two scaled)
#define SPLIT_DATA_RANGE 64.f

// ------------------------------------------------------------------------------------------------
// fp32 GEMMs on fp16 MFMA at fp32 accuracy ("3 x fp16 split", exponent-shifted):
//   w = w_h + w_l, d = d_h + d_l with fp16 halves; w.d ~= w_h.d_h + w_h.d_l + w_l.d_h (the dropped
//   w_l.d_l is <= 2^-22 relative).  A plain fp16 lo half (|lo| ~ 2^-11 |v|) is subnormal below
//   |v| ~ 2^-3 and loses bits there, so both lo halves are carried scaled by C = 2^SPLIT_SHIFT
//   and the whole product is accumulated at scale C:
//     weight side (2 fragments)  h  = fp16(w),       cl = fp16(C (w - h))
//     data side   (3 fragments)  ch = fp16(C d),     cl = fp16(C d - ch),    h = fp16(d)
//     C w.d ~= ch.h_w + h.cl_w + cl.h_w          (three v_mfma_f32_32x32x16_f16)
//   and the consumer multiplies the accumulator by 1/C (folded into its bias fma / flush scale).
//   Every fragment is a normal fp16 number for |w|, |d| >= 2^-2 / C (2.4e-4), so the relative
//   error per product stays at the fp32 level down there; below it the absolute error is
//   <= 2^-25 / C.  Range: |d| < 65504 / C (64; the reference's features stay below 10.4), |w| <
//   65504: an fp16 overflow makes the accumulator non-finite; kernels using this check it and
//   hand the launch to their exact-fp32 twin (Args::guard).  Three v_mfma_f32_32x32x16_f16 (32
//   cycles each) per 16 of K replace eight v_mfma_f32_32x32x2_f32 (64 cycles each).
// ------------------------------------------------------------------------------------------------
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f32x8 __attribute__((ext_vector_type(8)));

#define SPLIT_SHIFT 10
#define SPLIT_C 1024.0f
#define SPLIT_INV_C (1.0f / 1024.0f)

struct SplitW { h8 h, cl; };       // weight side: fp16(w), fp16(C (w - h))
struct SplitD { h8 ch, cl, h; };   // data side:   fp16(C d), fp16(C d - ch), fp16(d)

__device__ __forceinline__ SplitW split_w8(f32x8 v) {
  SplitW r;
  r.h = __builtin_convertvector(v, h8);
  r.cl = __builtin_convertvector((v - __builtin_convertvector(r.h, f32x8)) * SPLIT_C, h8);
  return r;
}

__device__ __forceinline__ SplitD split_d8(f32x8 v) {
  SplitD r;
  const f32x8 s = v * SPLIT_C;
  r.ch = __builtin_convertvector(s, h8);
  r.cl = __builtin_convertvector(s - __builtin_convertvector(r.ch, f32x8), h8);
  r.h = __builtin_convertvector(v, h8);
  return r;
}

// Power-of-two scale s with m s in [2^t, 2^(t+1)) (1 for m == 0 or a non-finite m): applied to a
// weight-side operand before split_w8 (per MFMA column, e.g. one W1 column) so its largest value
// sits near 2^t and its small values keep normal fp16 hi halves (a plain fp16 hi is subnormal
// below 6.1e-5, where 28 % of an L2 = 0.1 checkpoint's W1 lies); the consumer unscales by 1/s.
__device__ __forceinline__ float pow2_scale(float m, int t) {
  if (!(m > 0.f) || !(m <= 3.0e38f)) return 1.f;
  int e;
  frexpf(m, &e);  // m = f 2^e, f in [0.5, 1)
  e = e > 100 ? 100 : (e < -100 ? -100 : e);
  return ldexpf(1.f, t + 1 - e);
}

// acc += C (D.W) with the data fragments as the MFMA A operand (rows) and the weights as B
__device__ __forceinline__ f32x16 mfma3_dw(const SplitD& d, const SplitW& w, f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(d.cl, w.h, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(d.h, w.cl, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(d.ch, w.h, acc, 0, 0, 0);
}
// acc += C (W.D) with the weights as the A operand and the data fragments as B
__device__ __forceinline__ f32x16 mfma3_wd(const SplitW& w, const SplitD& d, f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(w.h, d.cl, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(w.cl, d.h, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(w.h, d.ch, acc, 0, 0, 0);
}

__device__ __forceinline__ float sum16(const f32x16& a) {
  float s0 = (a[0] + a[1]) + (a[2] + a[3]), s1 = (a[4] + a[5]) + (a[6] + a[7]);
  float s2 = (a[8] + a[9]) + (a[10] + a[11]), s3 = (a[12] + a[13]) + (a[14] + a[15]);
  return (s0 + s1) + (s2 + s3);
}

// hpe_set_exact_fp32(): 1 = exact-fp32 MFMA kernels only (hpe_rowprog.hip)
bool hpe_exact_fp32();

// hpe_kernel_timing(): HIP events around each program launch's dominant kernel (the fp16-split
// kernel, not its early-exit exact twin), recorded on the launch stream (hpe_rowprog.hip)
int hpe_tev_begin(hipStream_t s);
void hpe_tev_end(hipStream_t s, int slot);

// fused 2-layer regressor kernel (hpe_mlp2.hip)
int mlp2_supported(const int* words);
int mlp2_grid_cap(const int* words, int n_cu);
int mlp2_launch(const int* words_host, const Args& a, int grid, hipStream_t s);

// fused narrow chain forward (hpe_chain.hip)
int chain_supported(const int* words);
int chain_grid_cap(int n_cu);
int chain_lds_bytes();
int chain_launch(const int* words_host, const Args& a, int grid, hipStream_t s);

// fused residual-stack training (hpe_res.hip)
int res_supported(const int* words);
int res_grid_cap(int n_cu);
int res_launch(const int* words_host, const Args& a, int grid, hipStream_t s);
int res_fit_launch(const int* w, const int* dwords, float* params, float* params_t, float* m, float* v,
                   const float* l2, const int32_t* tpos, const float* x, const float* y_true, const int32_t* perm,
                   int64_t n, int32_t batch, int32_t kind, float beta_1, float beta_2, float epsilon,
                   const float* alpha, uint64_t seed_base, int64_t iter0, float* stats, int32_t stats_stride,
                   void* workspace, hipStream_t s);

// a program's word stream: host copy (kernel geometry) and device copy (kernel argument)
struct hpe_program;
const int* hpe_prog_words(const hpe_program* p);
const int* hpe_prog_dwords(const hpe_program* p);

// thread-local error message of the C ABI (hpe_last_error); returns code
int hpe_fail(int code, const char* fmt, ...);
