// hpe_blaze.hip — BlazeFace backbone forward: the frozen detector front of the
// unified models (BlazePoser/UnifiedModels/*.h5, run at blazeFaceDetectorH5.py:272), batched.
//
//   stem   conv 5x5 s2 'same' 3->24 + ReLU                       bf_stem_kernel
//   x16    DepthwiseConv2D 3x3 (s1|s2, TF 'same') -> 1x1 conv -> + residual (identity, or
//          MaxPool 2x2 s2) zero-padded in channels -> ReLU         bf_block_kernel<S, DW=1, NC>
//   heads  1x1 convs on the two taps (re_lu_10 16x16x88, re_lu_15 8x8x96), pairs fused into one
//          GEMM whose epilogue splits the channels into the two outputs  bf_block_kernel<1, 0, NC>
//
// Every op is one fused kernel: the input tile (+ halo) is staged HBM -> LDS once; each wave owns
// 32 output positions and computes the depthwise result just in time, in registers, as the A
// operand of v_mfma_f32_32x32x2_f32 (lane = position, k = channel, 4 channels per ds_read_b128 per
// tap), so the depthwise output never exists in memory; the pointwise weights (W^T) sit in LDS and
// the epilogue adds bias + residual (read back from the staged tile) + ReLU and writes NHWC.
// fp32 throughout (exact-f32 MFMA): per-op HBM traffic = input + output, the depthwise layers'
// 1.9 FLOP/B make the chain HBM-bound.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/hpe.h"
#include "hpe_common.h"

struct BfArgs {
  int f[BFO_WORDS];
  const float* params;
  const float* src;
  float* dst;
  float* dst2;
  int64_t nimg;
  int nwg;
};

__device__ __forceinline__ f32x4 ld4(const float* p) { return *(const f32x4*)p; }

// XCD-aware work id: consecutive work ids (the tiles of one image, whose halos overlap) stay on
// one XCD's L2 (hardware dispatches workgroups round-robin over the 8 XCDs).
__device__ __forceinline__ int xcd_work_id(int nwg) {
  const int b = blockIdx.x;
  if (nwg % 8) return b;
  return (b & 7) * (nwg >> 3) + (b >> 3);
}

// ------------------------------------------------------------------------------------------------
// stem: 5x5 s2 conv, TF 'same' on 128x128 (pad 1 top/left, 2 bottom/right), 3 -> 24, ReLU.
// K = (ky, kx, c) over a 6-row window (row 5 has zero weights) split by rows between the two lane
// halves (half h: ky = 3h + 0..2), so a lane's LDS offset for step s is base + const(s).
// ------------------------------------------------------------------------------------------------
#define STEM_KS 45
__global__ void __launch_bounds__(256) bf_stem_kernel(BfArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int* f = a.f;
  const int H = f[BFO_H], W = f[BFO_W], Wo = f[BFO_WO], Ho = f[BFO_HO];
  const int TH = f[BFO_TH], ROWS = f[BFO_ROWS], COLS = f[BFO_COLS];
  const int Cout = f[BFO_COUT];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, half = lane >> 5, l32 = lane & 31;
  const int tpi = Ho / TH;
  const int wid = xcd_work_id(a.nwg);
  const int64_t img = wid / tpi;
  const int oy0 = (wid % tpi) * TH;
  const float* P_ = a.params;
  // weights: W^T padded [32][90] (k = (ky*5 + kx)*3 + c, ky < 6), lane n = l32, its half's 45 k
  float wr[STEM_KS];
#pragma unroll
  for (int s = 0; s < STEM_KS; ++s) wr[s] = P_[f[BFO_PWW] + l32 * 90 + half * STEM_KS + s];
  // image tile rows iy = 2*oy0 - 1 + r, cols ix = c - 1, channel stride 3
  const int iy0 = oy0 * 2 - f[BFO_PADT];
  const int nflt = ROWS * COLS * 3;
  for (int e = threadIdx.x; e < nflt; e += blockDim.x) {
    const int r = e / (COLS * 3), rem = e - r * COLS * 3;
    const int c = rem / 3, ch = rem - c * 3;
    const int iy = iy0 + r, ix = c - f[BFO_PADL];
    float v = 0.f;
    if (iy >= 0 && iy < H && ix >= 0 && ix < W && img < a.nimg) v = a.src[((img * H + iy) * W + ix) * 3 + ch];
    lds[e] = v;
  }
  __syncthreads();
  if (img >= a.nimg) return;
  const int npos = TH * Wo;
  const float bias = l32 < Cout ? P_[f[BFO_PWB] + l32] : 0.f;
  for (int chunk = wave; chunk * 32 < npos; chunk += blockDim.x >> 6) {
    const int p = chunk * 32 + l32;
    const int oyl = p / Wo, ox = p - oyl * Wo;
    const float* t = lds + ((oyl * 2 + half * 3) * COLS + ox * 2) * 3;
    f32x16 acc = {};
#pragma unroll
    for (int s = 0; s < STEM_KS; ++s) {
      const int kyl = s / 15, kx = (s / 3) % 5, c = s % 3;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(t[(kyl * COLS + kx) * 3 + c], wr[s], acc, 0, 0, 0);
    }
    if (l32 < Cout) {
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int q = chunk * 32 + (g & 3) + 8 * (g >> 2) + 4 * half;
        const int qy = q / Wo, qx = q - qy * Wo;
        const float v = acc[g] + bias;
        a.dst[((img * Ho + oy0 + qy) * Wo + qx) * Cout + l32] = v > 0.f ? v : 0.f;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// block: [depthwise 3x3 (S, TF 'same') ->] 1x1 conv (MFMA) -> + residual -> [ReLU]
// LDS: W^T [NC*32][KS] | depthwise taps [9][Cinp] + bias [Cinp] | tile [NI][ROWS][COLS][CS]
// ------------------------------------------------------------------------------------------------
template <int S, int DW, int NC>
__global__ void __launch_bounds__(256) bf_block_kernel(BfArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int* f = a.f;
  const int H = f[BFO_H], W = f[BFO_W], Ho = f[BFO_HO], Wo = f[BFO_WO];
  const int Cinp = f[BFO_CINP], Cout = f[BFO_COUT], Coutp = f[BFO_COUTP];
  const int TH = f[BFO_TH], NI = f[BFO_NI], ROWS = f[BFO_ROWS], COLS = f[BFO_COLS];
  const int CS = f[BFO_CS], KS = f[BFO_KS], padt = f[BFO_PADT], padl = f[BFO_PADL];
  const int res = f[BFO_RES], relu = f[BFO_RELU], split = f[BFO_SPLIT], ostride = f[BFO_OSTRIDE];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, half = lane >> 5, l32 = lane & 31;
  const float* P_ = a.params;
  float* wt = lds;
  float* dwt = wt + NC * 32 * KS;
  float* tile = dwt + (DW ? 10 * Cinp : 0);

  const int tpi = Ho / TH;
  const int wid = xcd_work_id(a.nwg);
  const int64_t img0 = NI > 1 ? (int64_t)wid * NI : wid / tpi;
  const int oy0 = NI > 1 ? 0 : (wid % tpi) * TH;

  // ---- stage W^T (rows >= Coutp zero), depthwise table, input tile (zero outside the image) ----
  const int kq = Cinp >> 2;
  for (int i = threadIdx.x; i < NC * 32 * kq; i += blockDim.x) {
    const int n = i / kq, q = i - n * kq;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (n < Coutp) v = ld4(P_ + f[BFO_PWW] + n * Cinp + 4 * q);
    *(f32x4*)(wt + n * KS + 4 * q) = v;
  }
  if (DW)
    for (int i = threadIdx.x; i < 10 * kq; i += blockDim.x) *(f32x4*)(dwt + 4 * i) = ld4(P_ + f[BFO_DWW] + 4 * i);
  const int iy0 = oy0 * S - padt;
  const int per_img = ROWS * COLS * kq;
  for (int i = threadIdx.x; i < NI * per_img; i += blockDim.x) {
    const int il = i / per_img, rem = i - il * per_img;
    const int r = rem / (COLS * kq), rem2 = rem - r * COLS * kq;
    const int c = rem2 / kq, q = rem2 - c * kq;
    const int iy = iy0 + r, ix = c - padl;
    const int64_t img = img0 + il;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (iy >= 0 && iy < H && ix >= 0 && ix < W && img < a.nimg)
      v = ld4(a.src + ((img * H + iy) * W + ix) * Cinp + 4 * q);
    *(f32x4*)(tile + ((il * ROWS + r) * COLS + c) * CS + 4 * q) = v;
  }
  __syncthreads();

  const int ppi = TH * Wo;  // output positions per image in this tile
  const int npos = NI * ppi;
  const int nwaves = blockDim.x >> 6;
  for (int chunk = wave; chunk * 32 < npos; chunk += nwaves) {
    const int p = chunk * 32 + l32;
    const int il = p / ppi, pr = p - il * ppi;
    const int oyl = pr / Wo, ox = pr - oyl * Wo;
    const float* tb = tile + ((il * ROWS + oyl * S) * COLS + ox * S) * CS;
    f32x16 acc[NC];
#pragma unroll
    for (int nc = 0; nc < NC; ++nc) acc[nc] = (f32x16){};
    for (int c0 = 4 * half; c0 < Cinp; c0 += 8) {
      f32x4 av;
      if (DW) {
        av = ld4(dwt + 9 * Cinp + c0);
#pragma unroll
        for (int tp = 0; tp < 9; ++tp) {
          const f32x4 xv = ld4(tb + ((tp / 3) * COLS + (tp % 3)) * CS + c0);
          const f32x4 wv = ld4(dwt + tp * Cinp + c0);
          av.x = fmaf(xv.x, wv.x, av.x);
          av.y = fmaf(xv.y, wv.y, av.y);
          av.z = fmaf(xv.z, wv.z, av.z);
          av.w = fmaf(xv.w, wv.w, av.w);
        }
      } else {
        av = ld4(tb + c0);
      }
#pragma unroll
      for (int nc = 0; nc < NC; ++nc) {
        const f32x4 bv = ld4(wt + (nc * 32 + l32) * KS + c0);
        acc[nc] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.x, bv.x, acc[nc], 0, 0, 0);
        acc[nc] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.y, bv.y, acc[nc], 0, 0, 0);
        acc[nc] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.z, bv.z, acc[nc], 0, 0, 0);
        acc[nc] = __builtin_amdgcn_mfma_f32_32x32x2f32(av.w, bv.w, acc[nc], 0, 0, 0);
      }
    }
    // ---- epilogue: lane = output channel n, registers = 16 positions of the chunk ----
#pragma unroll
    for (int nc = 0; nc < NC; ++nc) {
      const int n = nc * 32 + l32;
      if (n >= Coutp) continue;
      const float bias = P_[f[BFO_PWB] + n];
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int q = chunk * 32 + (g & 3) + 8 * (g >> 2) + 4 * half;
        const int ql = q / ppi, qr = q - ql * ppi;
        const int qy = qr / Wo, qx = qr - qy * Wo;
        float v = acc[nc][g] + bias;
        if (res == BF_RES_ID) {
          if (n < Cinp) v += tile[((ql * ROWS + qy + padt) * COLS + qx + padl) * CS + n];
        } else if (res == BF_RES_MAXPOOL) {
          if (n < Cinp) {
            const float* t = tile + ((ql * ROWS + 2 * qy) * COLS + 2 * qx) * CS + n;
            v += fmaxf(fmaxf(t[0], t[CS]), fmaxf(t[COLS * CS], t[(COLS + 1) * CS]));
          }
        }
        if (relu) v = v > 0.f ? v : 0.f;
        const int64_t img = img0 + ql;
        if (img >= a.nimg) continue;
        const int64_t pos = (img * Ho + oy0 + qy) * Wo + qx;
        if (split) {
          if (n < split) a.dst[pos * split + n] = v;
          else if (n < Cout) a.dst2[pos * (Cout - split) + (n - split)] = v;
        } else if (n < ostride) {
          a.dst[pos * ostride + n] = v;
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
typedef void (*bf_fn)(BfArgs);

static bf_fn pick_block(int s, int dw, int nc) {
#define BF_NC(S_, DW_)                                   \
  switch (nc) {                                          \
    case 1: return bf_block_kernel<S_, DW_, 1>;          \
    case 2: return bf_block_kernel<S_, DW_, 2>;          \
    case 3: return bf_block_kernel<S_, DW_, 3>;          \
    case 4: return bf_block_kernel<S_, DW_, 4>;          \
    default: return nullptr;                             \
  }
  if (s == 1 && dw) { BF_NC(1, 1) }
  if (s == 2 && dw) { BF_NC(2, 1) }
  if (s == 1 && !dw) { BF_NC(1, 0) }
#undef BF_NC
  return nullptr;
}

struct hpe_blazeface {
  int* words;
  int n_words;
  int nops;
  int64_t act_floats;
};

static int check_op(const int* f, int i) {
  const int kind = f[BFO_KIND];
  if (kind != BF_STEM && kind != BF_BLOCK) return hpe_fail(HPE_EINVAL, "blazeface op %d: bad kind %d", i, kind);
  if (f[BFO_TH] <= 0 || f[BFO_NI] <= 0 || f[BFO_HO] % f[BFO_TH]) return hpe_fail(HPE_EINVAL, "blazeface op %d: bad tile", i);
  if ((f[BFO_NI] * f[BFO_TH] * f[BFO_WO]) % 32) return hpe_fail(HPE_EINVAL, "blazeface op %d: tile not a multiple of 32 positions", i);
  if (f[BFO_NI] > 1 && f[BFO_TH] != f[BFO_HO]) return hpe_fail(HPE_EINVAL, "blazeface op %d: multi-image tiles must be whole images", i);
  if (f[BFO_LDS] <= 0 || f[BFO_LDS] > 160 * 1024) return hpe_fail(HPE_EINVAL, "blazeface op %d: LDS %d bytes", i, f[BFO_LDS]);
  if (f[BFO_SRC] < 0 || f[BFO_SRC] >= BF_NBUF || f[BFO_DST] < 0 || f[BFO_DST] >= BF_NBUF)
    return hpe_fail(HPE_EINVAL, "blazeface op %d: bad buffer", i);
  if (kind == BF_STEM) {
    if (f[BFO_CIN] != 3 || f[BFO_COUT] > 32 || f[BFO_STRIDE] != 2) return hpe_fail(HPE_EINVAL, "blazeface stem: unsupported geometry");
    const int rows = 2 * (f[BFO_TH] - 1) + 6, cols = 2 * (f[BFO_WO] - 1) + 5;
    if (f[BFO_ROWS] != rows || f[BFO_COLS] != cols || f[BFO_LDS] < rows * cols * 12)
      return hpe_fail(HPE_EINVAL, "blazeface stem: tile words inconsistent");
    return 0;
  }
  const int s = f[BFO_STRIDE], dw = f[BFO_DW];
  if (!pick_block(s, dw, f[BFO_NC])) return hpe_fail(HPE_EINVAL, "blazeface op %d: no kernel for S=%d DW=%d NC=%d", i, s, dw, f[BFO_NC]);
  if (f[BFO_CINP] % 8 || f[BFO_CINP] < f[BFO_CIN] || f[BFO_COUTP] % 8 || f[BFO_COUTP] < f[BFO_COUT] ||
      f[BFO_NC] * 32 < f[BFO_COUTP] || f[BFO_CS] < f[BFO_CINP] || f[BFO_CS] % 4 || f[BFO_KS] < f[BFO_CINP] || f[BFO_KS] % 4)
    return hpe_fail(HPE_EINVAL, "blazeface op %d: channel geometry", i);
  const int rows = dw ? (f[BFO_TH] - 1) * s + 3 : f[BFO_TH];
  const int cols = dw ? (f[BFO_WO] - 1) * s + 3 : f[BFO_WO];
  if (f[BFO_ROWS] != rows || f[BFO_COLS] != cols) return hpe_fail(HPE_EINVAL, "blazeface op %d: tile rows/cols", i);
  if (f[BFO_RES] == BF_RES_MAXPOOL && (s != 2 || f[BFO_H] % 2 || f[BFO_W] % 2 || f[BFO_PADT] || f[BFO_PADL]))
    return hpe_fail(HPE_EINVAL, "blazeface op %d: maxpool residual needs s2 on even maps", i);
  if (f[BFO_RES] == BF_RES_ID && s != 1) return hpe_fail(HPE_EINVAL, "blazeface op %d: identity residual needs s1", i);
  const long need = 4L * (f[BFO_NC] * 32 * f[BFO_KS] + (dw ? 10 * f[BFO_CINP] : 0) +
                          (long)f[BFO_NI] * rows * cols * f[BFO_CS]);
  if (f[BFO_LDS] < need) return hpe_fail(HPE_EINVAL, "blazeface op %d: LDS words %d < %ld", i, f[BFO_LDS], need);
  if (!f[BFO_SPLIT] && (f[BFO_OSTRIDE] < f[BFO_COUT] || f[BFO_OSTRIDE] > f[BFO_COUTP]))
    return hpe_fail(HPE_EINVAL, "blazeface op %d: output stride", i);
  if (f[BFO_SPLIT] && (f[BFO_DST2] < 0 || f[BFO_DST2] >= BF_NBUF || f[BFO_SPLIT] >= f[BFO_COUT]))
    return hpe_fail(HPE_EINVAL, "blazeface op %d: bad split", i);
  return 0;
}

extern "C" int hpe_blazeface_create(const int32_t* words, int64_t n_words, hpe_blazeface** out) {
  if (!words || !out || n_words < BFH_WORDS) return hpe_fail(HPE_EINVAL, "blazeface: null/short words");
  if (words[BFH_MAGIC] != HPE_BF_MAGIC) return hpe_fail(HPE_EINVAL, "blazeface: bad magic");
  const int nops = words[BFH_NOPS], off = words[BFH_OPS_OFF];
  if (nops <= 0 || off < BFH_WORDS || off + (int64_t)nops * BFO_WORDS > n_words) return hpe_fail(HPE_EINVAL, "blazeface: bad op table");
  for (int i = 0; i < nops; ++i) {
    const int rc = check_op(words + off + i * BFO_WORDS, i);
    if (rc) return rc;
  }
  hpe_blazeface* h = (hpe_blazeface*)calloc(1, sizeof(hpe_blazeface));
  h->words = (int*)malloc(sizeof(int) * n_words);
  memcpy(h->words, words, sizeof(int) * n_words);
  h->n_words = (int)n_words;
  h->nops = nops;
  h->act_floats = words[BFH_ACT_FLOATS];
  *out = h;
  return HPE_OK;
}

extern "C" int hpe_blazeface_destroy(hpe_blazeface* h) {
  if (h) {
    free(h->words);
    free(h);
  }
  return HPE_OK;
}

extern "C" size_t hpe_blazeface_workspace_size(const hpe_blazeface* h, int64_t n_images) {
  if (!h || n_images <= 0) return 0;
  return (size_t)2 * (size_t)h->act_floats * (size_t)n_images * sizeof(float);
}

extern "C" int hpe_blazeface_forward(const hpe_blazeface* h, const float* params, const float* images,
                                     int64_t n_images, float* const* outs, void* workspace, void* stream) {
  if (!h || !params || !images || !outs || !workspace) return hpe_fail(HPE_EINVAL, "blazeface_forward: null argument");
  if (n_images <= 0) return HPE_OK;
  hipStream_t s = (hipStream_t)stream;
  float* bufs[BF_NBUF];
  bufs[BF_BUF_IMG] = (float*)images;
  bufs[BF_BUF_A] = (float*)workspace;
  bufs[BF_BUF_B] = (float*)workspace + h->act_floats * n_images;
  for (int i = 0; i < 6; ++i) {
    if (!outs[i]) return hpe_fail(HPE_EINVAL, "blazeface_forward: output %d is null", i);
    bufs[BF_BUF_OUT0 + i] = outs[i];
  }
  const int* ops = h->words + h->words[BFH_OPS_OFF];
  for (int i = 0; i < h->nops; ++i) {
    const int* f = ops + i * BFO_WORDS;
    BfArgs a;
    memcpy(a.f, f, sizeof a.f);
    a.params = params;
    a.src = bufs[f[BFO_SRC]];
    a.dst = bufs[f[BFO_DST]];
    a.dst2 = f[BFO_SPLIT] ? bufs[f[BFO_DST2]] : nullptr;
    a.nimg = n_images;
    const int64_t tpi = f[BFO_HO] / f[BFO_TH];
    const int64_t nwg = f[BFO_NI] > 1 ? (n_images + f[BFO_NI] - 1) / f[BFO_NI] : n_images * tpi;
    if (nwg > 0x7fffffff) return hpe_fail(HPE_EINVAL, "blazeface_forward: batch too large");
    a.nwg = (int)nwg;
    const int npos = f[BFO_NI] * f[BFO_TH] * f[BFO_WO];
    const int chunks = npos / 32;
    const int threads = 64 * (chunks < 4 ? chunks : 4);
    bf_fn k = f[BFO_KIND] == BF_STEM ? bf_stem_kernel : pick_block(f[BFO_STRIDE], f[BFO_DW], f[BFO_NC]);
    hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, f[BFO_LDS]);
    hipLaunchKernelGGL(k, dim3((unsigned)nwg), dim3(threads), f[BFO_LDS], s, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hpe_fail(HPE_ERUNTIME, "blazeface op %d launch: %s", i, hipGetErrorString(e));
  }
  return HPE_OK;
}
