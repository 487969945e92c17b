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
// tap; fp16-split MFMA, see mfma_split), so the depthwise output never exists in memory; the
// pointwise weights (W^T, as fp16 hi/lo pairs) sit in LDS and
// the epilogue adds bias + residual (read back from the staged tile) + ReLU and writes NHWC.
// fp32 arithmetic throughout (every GEMM as fp16 MFMA products at fp32 accuracy): per-op HBM traffic =
// input + output, the depthwise layers' 1.9 FLOP/B make the chain HBM-bound.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/hpe.h"
#include "hpe_common.h"
#include "hpe_dev.h"

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

// Pointwise convs on fp16 MFMA (configs[4]: "fp16 MFMA on pointwise convs") at fp32 accuracy:
// a = a_hi + a_lo, b = b_hi + b_lo with fp16 halves, a.b ~= a_hi.b_hi + a_hi.b_lo + a_lo.b_hi
// (dropped a_lo.b_lo ~ 2^-22 relative), fp32 accumulate: three v_mfma_f32_32x32x8_f16 per 8
// channels replace four v_mfma_f32_32x32x2_f32 (64 cycles each) per 8 channels.  The W^T table
// holds each quad of weights as {hi[4], lo[4]} (16 B, the footprint of the fp32 quad it replaces).
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ h4 to_h4(f32x4 v) {
  return h4{(_Float16)v.x, (_Float16)v.y, (_Float16)v.z, (_Float16)v.w};
}
__device__ __forceinline__ f32x4 split_w(f32x4 v) {  // fp32 quad -> packed {hi[4], lo[4]}
  const h4 hi = to_h4(v);
  const h4 lo = to_h4(v - f32x4{(float)hi.x, (float)hi.y, (float)hi.z, (float)hi.w});
  h8 r = {hi.x, hi.y, hi.z, hi.w, lo.x, lo.y, lo.z, lo.w};
  return *(f32x4*)&r;
}
__device__ __forceinline__ f32x16 mfma_split(f32x4 av, f32x4 wpk, f32x16 acc) {
  const h4 ah = to_h4(av);
  const h4 al = to_h4(av - f32x4{(float)ah.x, (float)ah.y, (float)ah.z, (float)ah.w});
  const h8 w = *(const h8*)&wpk;
  const h4 bh = {w[0], w[1], w[2], w[3]}, bl = {w[4], w[5], w[6], w[7]};
  acc = __builtin_amdgcn_mfma_f32_32x32x8f16(al, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x8f16(ah, bl, acc, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x8f16(ah, bh, acc, 0, 0, 0);
}

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
// halves (half h: ky = 3h + 0..2, 45 k each, padded to 48), so a lane's LDS offset for k is its
// base + a compile-time constant.  The GEMM runs on fp16 MFMA at fp32 accuracy (the exponent-shifted
// 3-product split of hpe_common.h, six K-steps of v_mfma_f32_32x32x16_f16 x 3 = 18 MFMAs of 32
// cycles per 32 positions instead of 45 fp32 v_mfma_f32_32x32x2_f32 of 64): weights scaled per
// output channel by a power of two (pow2_scale), data = the preprocessed frame, |x| <= 1 in the
// reference ((x - 0.5) / 0.5, blazeFaceDetectorH5.py:244-269; the split's data range is |x| < 64).
// ------------------------------------------------------------------------------------------------
#define STEM_KS 45
#define STEM_NK 6   // K-steps of 8 k per lane half
__global__ void __launch_bounds__(256) bf_stem_kernel(BfArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int* f = a.f;
  const int H = f[BFO_H], W = f[BFO_W], Wo = f[BFO_WO], Ho = f[BFO_HO];
  const int TH = f[BFO_TH], ROWS = f[BFO_ROWS], COLS = f[BFO_COLS];
  const int Cout = f[BFO_COUT];
  const int lgWo = __builtin_ctz(Wo);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, half = lane >> 5, l32 = lane & 31;
  const int tpi = Ho / TH;
  const int wid = xcd_work_id(a.nwg);
  const int64_t img = wid / tpi;
  const int oy0 = (wid - (int)img * tpi) * TH;
  const float* P_ = a.params;
  // weights: W^T padded [32][90] (k = (ky*5 + kx)*3 + c, ky < 6), lane n = l32, its half's 45 k as
  // split fragments of K-step s = k-local 8 s .. 8 s + 7, scaled by s1 (max |w| of the channel in
  // [2^13, 2^14)); z = acc * inv + bias, inv = 1 / (C s1)
  SplitW wsp[STEM_NK];
  float inv;
  {
    f32x8 v[STEM_NK];
    float mx = 0.f;
#pragma unroll
    for (int s = 0; s < STEM_NK; ++s) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int q = 8 * s + j;
        v[s][j] = q < STEM_KS ? P_[f[BFO_PWW] + l32 * 90 + half * STEM_KS + q] : 0.f;
        mx = fmaxf(mx, fabsf(v[s][j]));
      }
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float s1 = pow2_scale(mx, 13);
    inv = SPLIT_INV_C / s1;
#pragma unroll
    for (int s = 0; s < STEM_NK; ++s) wsp[s] = split_w8(v[s] * s1);
  }
  // image tile: LDS row r <-> image row 2*oy0 - padt + r; a row is W*3 contiguous floats placed at
  // column padl (zeros around), no per-element division
  const int iy0 = oy0 * 2 - f[BFO_PADT];
  const int padl3 = f[BFO_PADL] * 3, rowf = COLS * 3, W3 = W * 3;
  // batches of 8 loads per thread, all issued (from clamped addresses) before the LDS writes
  const int nT = ROWS * rowf;
  for (int e0 = threadIdx.x; e0 < nT; e0 += 8 * blockDim.x) {
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int e = e0 + i * blockDim.x;
      const int r = e / rowf, x3 = e - r * rowf - padl3;
      const int iy = iy0 + r;
      const bool ok = e < nT && iy >= 0 && iy < H && x3 >= 0 && x3 < W3 && img < a.nimg;
      v[i] = a.src[ok ? (img * H + iy) * W * 3 + x3 : 0];
      if (!ok) v[i] = 0.f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int e = e0 + i * blockDim.x;
      if (e < nT) lds[e] = v[i];
    }
  }
  __syncthreads();
  if (img >= a.nimg) return;
  const int npos = TH * Wo;
  const float bias = l32 < Cout ? P_[f[BFO_PWB] + l32] : 0.f;
  for (int chunk = wave; chunk * 32 < npos; chunk += blockDim.x >> 6) {
    const int p = chunk * 32 + l32;
    const int oyl = p >> lgWo, ox = p & (Wo - 1);
    const float* t = lds + (oyl * 2 + half * 3) * rowf + ox * 6;
    f32x16 acc = {};
#pragma unroll
    for (int s = 0; s < STEM_NK; ++s) {
      f32x8 xv;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int q = 8 * s + j;   // compile-time: (ky - 3 half, kx, c) = (q / 15, q / 3 % 5, q % 3)
        xv[j] = q < STEM_KS ? t[(q / 15) * rowf + ((q / 3) % 5) * 3 + q % 3] : 0.f;
      }
      acc = mfma3_dw(split_d8(xv), wsp[s], acc);
    }
    if (l32 < Cout) {
      float* drow = a.dst + ((img * Ho + oy0) * Wo) * Cout + l32;
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int q = chunk * 32 + (g & 3) + 8 * (g >> 2) + 4 * half;   // q = qy * Wo + qx
        const float v = fmaf(acc[g], inv, bias);
        drow[q * Cout] = v > 0.f ? v : 0.f;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// block: [depthwise 3x3 (S, TF 'same') ->] 1x1 conv (MFMA) -> + residual -> [ReLU]
// LDS: W^T [NCT*32][KS] | depthwise taps [9][Cinp] + bias [Cinp] | tile [NI][ROWS][COLS][CS]
// A wave task is (32-position chunk, group of NC output-channel chunks of 32): the depthwise A
// operand is recomputed per group (cheap VALU next to the MFMA) to give every WG >= 4 waves.
// Wo and TH*Wo are powers of two (checked on the host), so position math is shifts.
// ------------------------------------------------------------------------------------------------
template <int S, int DW, int NC>
__global__ void __launch_bounds__(512) bf_block_kernel(BfArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int* f = a.f;
  const int H = f[BFO_H], W = f[BFO_W], Ho = f[BFO_HO], Wo = f[BFO_WO];
  const int Cinp = f[BFO_CINP], Cout = f[BFO_COUT], Coutp = f[BFO_COUTP];
  const int TH = f[BFO_TH], NI = f[BFO_NI], ROWS = f[BFO_ROWS], COLS = f[BFO_COLS];
  const int CS = f[BFO_CS], KS = f[BFO_KS], padt = f[BFO_PADT], padl = f[BFO_PADL];
  const int res = f[BFO_RES], relu = f[BFO_RELU], split = f[BFO_SPLIT], ostride = f[BFO_OSTRIDE];
  const int NCT = f[BFO_NCT];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, half = lane >> 5, l32 = lane & 31;
  const int lgWo = __builtin_ctz(Wo), lgP = __builtin_ctz(TH * Wo);
  const float* P_ = a.params;
  float* wt = lds;
  float* dwt = wt + NCT * 32 * KS;
  float* tile = dwt + (DW ? 10 * Cinp : 0);

  const int tpi = Ho / TH;
  const int wid = xcd_work_id(a.nwg);
  const int64_t img0 = NI > 1 ? (int64_t)wid * NI : wid / tpi;
  const int oy0 = NI > 1 ? 0 : (wid - (int)img0 * tpi) * TH;

  // ---- stage W^T (rows >= Coutp zero), depthwise table, input tile (zero outside the image) ----
  // batches of 8 float4 per thread: every load of a batch is issued (from a clamped, always valid
  // address) before the first LDS write, so a workgroup's staging costs ~one HBM round trip per
  // batch instead of one per element (a conditional load per element serialises on vmcnt(0))
  const int kq = Cinp >> 2;
  const int nthr = blockDim.x;
  {
    const int nW = NCT * 32 * kq;
    for (int e0 = threadIdx.x; e0 < nW; e0 += 8 * nthr) {
      f32x4 v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int e = e0 + i * nthr;
        const int n = e / kq, q = e - n * kq;
        const bool ok = e < nW && n < Coutp;
        v[i] = ld4(P_ + f[BFO_PWW] + (ok ? n * Cinp + 4 * q : 0));
        if (!ok) v[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int e = e0 + i * nthr;
        const int n = e / kq, q = e - n * kq;
        if (e < nW) *(f32x4*)(wt + n * KS + 4 * q) = split_w(v[i]);
      }
    }
    const int iy0 = oy0 * S - padt;
    const int nT = NI * ROWS * COLS * kq;
    for (int e0 = threadIdx.x; e0 < nT; e0 += 8 * nthr) {
      f32x4 v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int e = e0 + i * nthr;
        const int pix = e / kq, q = e - pix * kq;
        const int rr = pix / COLS, c = pix - rr * COLS;
        const int il = rr / ROWS, r = rr - il * ROWS;
        const int64_t img = img0 + il;
        const int iy = iy0 + r, ix = c - padl;
        const bool ok = e < nT && iy >= 0 && iy < H && ix >= 0 && ix < W && img < a.nimg;
        v[i] = ld4(a.src + (ok ? ((img * H + iy) * W + ix) * Cinp + 4 * q : 0));
        if (!ok) v[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int e = e0 + i * nthr;
        const int pix = e / kq, q = e - pix * kq;
        if (e < nT) *(f32x4*)(tile + pix * CS + 4 * q) = v[i];
      }
    }
  }
  if (DW)
    for (int i = threadIdx.x; i < 10 * kq; i += nthr) *(f32x4*)(dwt + 4 * i) = ld4(P_ + f[BFO_DWW] + 4 * i);
  __syncthreads();

  const int npos = NI * TH * Wo;
  const int ngrp = NCT / NC;
  const int ntask = (npos >> 5) * ngrp;
  const int nwaves = nthr >> 6;
  const int colsCS = COLS * CS;
  for (int task = wave; task < ntask; task += nwaves) {
    const int chunk = task / ngrp, grp = task - chunk * ngrp;
    const int p = chunk * 32 + l32;
    const int il = p >> lgP, pr = p & ((1 << lgP) - 1);
    const int oyl = pr >> lgWo, ox = pr & (Wo - 1);
    const float* tb = tile + (il * ROWS + oyl * S) * colsCS + ox * S * CS;
    const float* wb = wt + (grp * NC * 32 + l32) * KS;
    f32x16 acc[NC];
#pragma unroll
    for (int nc = 0; nc < NC; ++nc) acc[nc] = (f32x16){};
#pragma unroll 2
    for (int c0 = 4 * half; c0 < Cinp; c0 += 8) {
      f32x4 av;
      if (DW) {
        av = ld4(dwt + 9 * Cinp + c0);
#pragma unroll
        for (int tp = 0; tp < 9; ++tp) {
          const f32x4 xv = ld4(tb + (tp / 3) * colsCS + (tp % 3) * CS + c0);
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
        acc[nc] = mfma_split(av, ld4(wb + nc * 32 * KS + c0), acc[nc]);
      }
    }
    // ---- epilogue: lane = output channel n, registers = 16 positions of the chunk ----
#pragma unroll
    for (int nc = 0; nc < NC; ++nc) {
      const int n = (grp * NC + nc) * 32 + l32;
      if (n >= Coutp) continue;
      const float bias = P_[f[BFO_PWB] + n];
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int q = chunk * 32 + (g & 3) + 8 * (g >> 2) + 4 * half;
        const int ql = q >> lgP, qr = q & ((1 << lgP) - 1);
        const int qy = qr >> lgWo, qx = qr & (Wo - 1);
        float v = acc[nc][g] + bias;
        if (res == BF_RES_ID) {
          if (n < Cinp) v += tile[(ql * ROWS + qy + padt) * colsCS + (qx + padl) * CS + n];
        } else if (res == BF_RES_MAXPOOL) {
          if (n < Cinp) {
            const float* t = tile + (ql * ROWS + 2 * qy) * colsCS + 2 * qx * CS + n;
            v += fmaxf(fmaxf(t[0], t[CS]), fmaxf(t[colsCS], t[colsCS + CS]));
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
// rows: the same fused block, streamed.  A workgroup owns a segment of one image's output rows
// and walks it TH rows per step.  LDS holds W^T, the depthwise table and a ring of ROWS input
// rows (exactly the rows one step reads); the R*S input rows the next step adds are loaded into
// registers while this step computes (each thread's share is a contiguous run of the NHWC rows, so
// the loads are plain coalesced float4s), and written over the ring slots this step frees.  Every
// input byte is read from HBM once per segment: no halo tiles, no load/compute serialisation.
// ------------------------------------------------------------------------------------------------
#define RPF 4   // max float4 prefetched per thread per step

// CINP / COUTP > 0: channel counts fixed at compile time (every LDS offset of the depthwise taps,
// W^T rows and the epilogue becomes an immediate; the VALU work per step is then the depthwise FMAs
// and little else).  0: read from the op words.  Wo >= 16 (a power of two): a 32-position chunk is one output row, or two at Wo = 16.
template <int S, int NC_, int CINP, int COUTP>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) bf_rows_kernel(BfArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int NC = COUTP ? (COUTP + 31) / 32 : NC_;
  const int* f = a.f;
  const int H = f[BFO_H], W = f[BFO_W], Ho = f[BFO_HO], Wo = f[BFO_WO];
  const int Cinp = CINP ? CINP : f[BFO_CINP];
  const int Coutp = COUTP ? COUTP : f[BFO_COUTP];
  const int CS = CINP ? CINP + 4 : f[BFO_CS];
  const int KS = CINP ? CINP + 4 : f[BFO_KS];
  const int ostride = COUTP ? COUTP : f[BFO_OSTRIDE];
  const int NCT = COUTP ? NC : f[BFO_NCT];
  const int R = f[BFO_TH], NSEG = f[BFO_NI], RING = f[BFO_ROWS], COLS = f[BFO_COLS];
  const int padt = f[BFO_PADT], padl = f[BFO_PADL];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, half = lane >> 5, l32 = lane & 31;
  const int lgWo = __builtin_ctz(Wo);
  const int nthr = blockDim.x, nwaves = nthr >> 6;
  const float* P_ = a.params;
  float* wt = lds;
  float* dwt = wt + NCT * 32 * KS;
  float* ring = dwt + 10 * Cinp;
  const int rowLDS = COLS * CS;

  const int wid = xcd_work_id(a.nwg);
  const int64_t img = wid / NSEG;
  const int seg = wid - (int)img * NSEG;
  const int seg_rows = Ho / NSEG;
  const int oy_begin = seg * seg_rows;
  const int kq = Cinp >> 2;
  const float* simg = a.src + img * (int64_t)H * W * Cinp;

  // ---- W^T, depthwise table, zeroed ring (pad columns stay zero for the whole launch) ----
  for (int i = threadIdx.x; i < NCT * 32 * kq; i += nthr) {
    const int n = i / kq, q = i - n * kq;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (n < Coutp) v = split_w(ld4(P_ + f[BFO_PWW] + n * Cinp + 4 * q));
    *(f32x4*)(wt + n * KS + 4 * q) = v;
  }
  for (int i = threadIdx.x; i < 10 * kq; i += nthr) *(f32x4*)(dwt + 4 * i) = ld4(P_ + f[BFO_DWW] + 4 * i);
  for (int i = threadIdx.x; i < RING * rowLDS / 4; i += nthr) *(f32x4*)(ring + 4 * i) = (f32x4){0.f, 0.f, 0.f, 0.f};
  __syncthreads();

  // ---- prologue: the first step's RING input rows straight into the ring ----
  const int rowq = W * kq;  // float4 per input row (contiguous in HBM)
  {
    const int iy0 = oy_begin * S - padt;
    for (int e = threadIdx.x; e < RING * rowq; e += nthr) {
      const int rr = e / rowq, rem = e - rr * rowq;
      const int ix = rem / kq, q = rem - ix * kq;
      const int iy = iy0 + rr;
      if (iy >= 0 && iy < H) {
        const int slot = (iy + RING) % RING;
        *(f32x4*)(ring + slot * rowLDS + (ix + padl) * CS + 4 * q) = ld4(simg + ((int64_t)iy * W + ix) * Cinp + 4 * q);
      }
    }
  }
  // per-thread share of a step's new rows: float4 e = t + i*nthr of the NEW contiguous rows
  const int NEW = R * S;
  const int newq = NEW * rowq;
  int pf_row[RPF], pf_off[RPF];
#pragma unroll
  for (int i = 0; i < RPF; ++i) {
    const int e = threadIdx.x + i * nthr;
    const int rr = e / rowq, rem = e - rr * rowq;
    const int ix = rem / kq, q = rem - ix * kq;
    pf_row[i] = e < newq ? rr : -1;
    pf_off[i] = (ix + padl) * CS + 4 * q;
  }
  __syncthreads();

  const int ngrp = NCT / NC;
  const int ntask = ((R * Wo) >> 5) * ngrp;
  const int nsteps = seg_rows / R;

  auto compute = [&](int oy0) {
    for (int task = wave; task < ntask; task += nwaves) {
      const int chunk = task / ngrp, grp = task - chunk * ngrp;
      // a 32-position chunk covers one output row (Wo >= 32) or two (Wo = 16): row oyA, and oyA + 1
      // for positions past the row end; the lane's depthwise position is p0 + l32
      const int p0 = chunk * 32;
      const int oyA = oy0 + (p0 >> lgWo);
      const int pl = p0 + l32;
      const int oyl = oy0 + (pl >> lgWo), xl = pl & (Wo - 1);
      int s0 = oyl * S - padt;
      s0 = (s0 + RING) % RING;
      const int s1 = s0 + 1 == RING ? 0 : s0 + 1;
      const int s2 = s1 + 1 == RING ? 0 : s1 + 1;
      const int colx = xl * S * CS;
      const float* r0 = ring + s0 * rowLDS + colx;
      const float* r1 = ring + s1 * rowLDS + colx;
      const float* r2 = ring + s2 * rowLDS + colx;
      const float* wb = wt + (grp * NC * 32 + l32) * KS;
      f32x16 acc[NC];
#pragma unroll
      for (int nc = 0; nc < NC; ++nc) acc[nc] = (f32x16){};
#pragma unroll 1
      for (int c0 = 4 * half; c0 < (CINP ? CINP : Cinp); c0 += 8) {
        f32x4 av = ld4(dwt + 9 * Cinp + c0);
#pragma unroll
        for (int tp = 0; tp < 9; ++tp) {
          const float* rp = tp < 3 ? r0 : (tp < 6 ? r1 : r2);
          const f32x4 xv = ld4(rp + (tp % 3) * CS + c0);
          const f32x4 wv = ld4(dwt + tp * Cinp + c0);
          av.x = fmaf(xv.x, wv.x, av.x);
          av.y = fmaf(xv.y, wv.y, av.y);
          av.z = fmaf(xv.z, wv.z, av.z);
          av.w = fmaf(xv.w, wv.w, av.w);
        }
#pragma unroll
        for (int nc = 0; nc < NC; ++nc) {
          acc[nc] = mfma_split(av, ld4(wb + nc * 32 * KS + c0), acc[nc]);
        }
      }
      // epilogue: register g <-> step position q = p0 + 4*half + (g&3) + 8*(g>>2): output row
      // oy0 + (q >> lgWo) (oyA, or oyA + 1 when the chunk wraps), column q & (Wo - 1); the output
      // address is linear in q.  Residual rows of oyA / oyA + 1 in the ring:
      const float *rA, *rA1 = nullptr, *rB, *rB1 = nullptr;
      if (S == 1) {
        rA = ring + (oyA % RING) * rowLDS + padl * CS;
        rB = ring + ((oyA + 1) % RING) * rowLDS + padl * CS;
      } else {
        rA = ring + ((2 * oyA) % RING) * rowLDS;
        rA1 = ring + ((2 * oyA + 1) % RING) * rowLDS;
        rB = ring + ((2 * oyA + 2) % RING) * rowLDS;
        rB1 = ring + ((2 * oyA + 3) % RING) * rowLDS;
      }
      float* out = a.dst + ((img * Ho + oy0) * Wo + p0 + 4 * half) * ostride;
#pragma unroll
      for (int nc = 0; nc < NC; ++nc) {
        const int n = (grp * NC + nc) * 32 + l32;
        if (n >= Coutp) continue;
        const float bias = P_[f[BFO_PWB] + n];
        const bool has_res = n < Cinp;
#pragma unroll
        for (int g = 0; g < 16; ++g) {
          const int d = (g & 3) + 8 * (g >> 2);
          float v = acc[nc][g] + bias;
          if (has_res) {
            const int q = p0 + 4 * half + d;
            const bool second = (q >> lgWo) != (p0 >> lgWo);
            const int xg = q & (Wo - 1);
            if (S == 1) {
              v += (second ? rB : rA)[xg * CS + n];
            } else {
              const float* t0 = (second ? rB : rA) + 2 * xg * CS + n;
              const float* t1 = (second ? rB1 : rA1) + 2 * xg * CS + n;
              v += fmaxf(fmaxf(t0[0], t0[CS]), fmaxf(t1[0], t1[CS]));
            }
          }
          out[d * ostride + n] = v > 0.f ? v : 0.f;
        }
      }
    }
  };
  // first input row step j adds (rows of step j-1 plus NEW more); its NEW rows are contiguous in HBM
  auto first_new = [&](int j) { return (oy_begin + j * R) * S - padt + (RING - NEW); };
  auto issue = [&](f32x4 (&pf)[RPF], int j) {
    if (j >= nsteps) return;
    const int r0 = first_new(j);
    const float* base = simg + (int64_t)r0 * rowq * 4 + threadIdx.x * 4;
#pragma unroll
    for (int i = 0; i < RPF; ++i)
      if (pf_row[i] >= 0 && r0 + pf_row[i] < H) pf[i] = ld4(base + i * nthr * 4);
  };
  auto commit = [&](f32x4 (&pf)[RPF], int j) {
    const int r0 = first_new(j);
    const int slot0 = (r0 + RING) % RING;
#pragma unroll
    for (int i = 0; i < RPF; ++i) {
      if (pf_row[i] < 0) continue;
      int sl = slot0 + pf_row[i];
      sl -= sl >= RING ? RING : 0;
      const f32x4 v = r0 + pf_row[i] < H ? pf[i] : (f32x4){0.f, 0.f, 0.f, 0.f};
      *(f32x4*)(ring + sl * rowLDS + pf_off[i]) = v;
    }
  };
  // three steps of rows in flight per workgroup
  f32x4 pa[RPF], pb[RPF], pc[RPF];
  issue(pa, 1);
  issue(pb, 2);
  issue(pc, 3);
  for (int k = 0; k < nsteps; k += 3) {
    compute(oy_begin + k * R);
    __syncthreads();
    if (k + 1 >= nsteps) break;
    commit(pa, k + 1);
    issue(pa, k + 4);
    __syncthreads();
    compute(oy_begin + (k + 1) * R);
    __syncthreads();
    if (k + 2 >= nsteps) break;
    commit(pb, k + 2);
    issue(pb, k + 5);
    __syncthreads();
    compute(oy_begin + (k + 2) * R);
    __syncthreads();
    if (k + 3 >= nsteps) break;
    commit(pc, k + 3);
    issue(pc, k + 6);
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------------
// ------------------------------------------------------------------------------------------------
// direct: the fused block for the small maps (16x16, 8x8) and the detector heads.  Persistent
// workgroups keep W^T (fp16 hi/lo pairs) and the depthwise table in LDS for the whole launch; each
// wave task is a 32-position chunk of one image with ALL output-channel chunks (no depthwise
// recompute), its nine 3x3 taps read straight from global memory (the 9x reuse is served by
// L1 / L2, no tile staging, no workgroup barrier in the loop), residual from global, NHWC store.
// ------------------------------------------------------------------------------------------------
template <int S, int DW, int NC>
__global__ void __launch_bounds__(256) bf_direct_kernel(BfArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int* f = a.f;
  const int H = f[BFO_H], W = f[BFO_W], Wo = f[BFO_WO], Ho = f[BFO_HO];
  const int Cinp = f[BFO_CINP], Cout = f[BFO_COUT], Coutp = f[BFO_COUTP];
  const int KS = f[BFO_KS], padt = f[BFO_PADT], padl = f[BFO_PADL];
  const int res = f[BFO_RES], relu = f[BFO_RELU], split = f[BFO_SPLIT], ostride = f[BFO_OSTRIDE];
  const int NCT = f[BFO_NCT];
  const int lane = threadIdx.x & 63, half = lane >> 5, l32 = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lgWo = __builtin_ctz(Wo);
  const float* P_ = a.params;
  float* wt = lds;
  float* dwt = wt + NCT * 32 * KS;
  const int kq = Cinp >> 2;
  const int nthr = blockDim.x;
  {  // W^T (split) + depthwise table, batched loads
    const int nW = NCT * 32 * kq;
    for (int e0 = threadIdx.x; e0 < nW; e0 += 8 * nthr) {
      f32x4 v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int e = e0 + i * nthr;
        const int n = e / kq, q = e - n * kq;
        const bool ok = e < nW && n < Coutp;
        v[i] = ld4(P_ + f[BFO_PWW] + (ok ? n * Cinp + 4 * q : 0));
        if (!ok) v[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int e = e0 + i * nthr;
        const int n = e / kq, q = e - n * kq;
        if (e < nW) *(f32x4*)(wt + n * KS + 4 * q) = split_w(v[i]);
      }
    }
    if (DW)
      for (int i = threadIdx.x; i < 10 * kq; i += nthr) *(f32x4*)(dwt + 4 * i) = ld4(P_ + f[BFO_DWW] + 4 * i);
  }
  __syncthreads();

  const int cpi = (Ho * Wo) >> 5;
  const int64_t ntask = a.nimg * cpi;
  const int nwaves = nthr >> 6;
  const int64_t istride = (int64_t)H * W * Cinp;
  for (int64_t task = (int64_t)blockIdx.x * nwaves + wave; task < ntask; task += (int64_t)gridDim.x * nwaves) {
    const int64_t img = task / cpi;
    const int chunk = (int)(task - img * cpi);
    const float* xi = a.src + img * istride;
    const int p = chunk * 32 + l32;
    const int oy = p >> lgWo, ox = p & (Wo - 1);
    int toff[9];
    uint32_t tmask = 0;
#pragma unroll
    for (int tp = 0; tp < 9; ++tp) {
      const int iy = oy * S - padt + tp / 3, ix = ox * S - padl + tp % 3;
      const bool ok = DW ? (iy >= 0 && iy < H && ix >= 0 && ix < W) : tp == 4;
      toff[tp] = ok ? (iy * W + ix) * Cinp : 0;
      tmask |= ok ? (1u << tp) : 0u;
    }
    if (!DW) toff[4] = (oy * W + ox) * Cinp;
    f32x16 acc[NC];
#pragma unroll
    for (int nc = 0; nc < NC; ++nc) acc[nc] = (f32x16){};
#pragma unroll 2
    for (int c0 = 4 * half; c0 < Cinp; c0 += 8) {
      f32x4 av;
      if (DW) {
        f32x4 xv[9];
#pragma unroll
        for (int tp = 0; tp < 9; ++tp) xv[tp] = ld4(xi + toff[tp] + c0);
        av = ld4(dwt + 9 * Cinp + c0);
#pragma unroll
        for (int tp = 0; tp < 9; ++tp) {
          const f32x4 x = (tmask >> tp) & 1u ? xv[tp] : f32x4{0.f, 0.f, 0.f, 0.f};
          const f32x4 wv = ld4(dwt + tp * Cinp + c0);
          av.x = fmaf(x.x, wv.x, av.x);
          av.y = fmaf(x.y, wv.y, av.y);
          av.z = fmaf(x.z, wv.z, av.z);
          av.w = fmaf(x.w, wv.w, av.w);
        }
      } else {
        av = ld4(xi + toff[4] + c0);
      }
#pragma unroll
      for (int nc = 0; nc < NC; ++nc) acc[nc] = mfma_split(av, ld4(wt + (nc * 32 + l32) * KS + c0), acc[nc]);
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
        const int qy = q >> lgWo, qx = q & (Wo - 1);
        float v = acc[nc][g] + bias;
        if (res == BF_RES_ID) {
          if (n < Cinp) v += xi[(qy * W + qx) * Cinp + n];
        } else if (res == BF_RES_MAXPOOL) {
          if (n < Cinp) {
            const float* t = xi + ((2 * qy) * W + 2 * qx) * Cinp + n;
            v += fmaxf(fmaxf(t[0], t[Cinp]), fmaxf(t[W * Cinp], t[W * Cinp + Cinp]));
          }
        }
        if (relu) v = v > 0.f ? v : 0.f;
        const int64_t pos = (img * Ho + qy) * Wo + qx;
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


// one op of a stage (host-filled from its BFO record)
struct BfSub {
  int s, h, w, ho, wo, cin, cinp, cout, coutp, ks, nct, nc, res, relu, dw, padt, padl, dww, pww, pwb;
  int var;      // task variant (BFV_*), picked on the host
  int wto;      // this op's W^T at wt + wto (the band op keeps it clear of its staging rows)
  int sst;      // BFV_BAND: channel stride of the staged source rows
  int ss, cso;  // channel strides of the resident source map (cinp + 4) and of the output map
  int zhalo;    // 1: zero the output map's halo rows (its geometry differs from the source's)
  int lds_out;  // 1: the output map stays in LDS (blocks)
  int gdst, gdst2, split, ostride;  // global output buffer(s): taps (gdst), heads (split epilogue); -1 none
};
#define BFS_MAX 16
struct BfStageArgs {
  BfSub op[BFS_MAX];
  int nops, map_floats, wt_floats;
  const float* params;
  const float* src;
  float* bufs[BF_NBUF];
};

// ------------------------------------------------------------------------------------------------
// stage: the small-map tail of the backbone (every block from the first one whose output map has
// <= 256 positions, e.g. 32x32 -> 16x16 s2 onwards) and the detector heads, ONE workgroup per image,
// the activation map resident in LDS across all its layers.  The per-op kernels above read and
// write every intermediate map through HBM (16x16 and 8x8 maps: 0.12-0.24 of HBM bandwidth, each
// op's launch too short to fill the chip); here the only HBM traffic is the stage's input map,
// the two taps and the head outputs.
//   LDS: map [HW][CS] (in place: a block's outputs stay in registers until every wave has read
//        its inputs, one barrier, then overwrite them; a stride-2 block's smaller output overlays
//        the start of its input the same way) | W^T of the current op (fp16 hi/lo pairs) | dw table
//   per op: <= 8 wave tasks (32-position chunk x group of NC output-channel chunks of 32), the same
//        arithmetic as bf_block_kernel / bf_direct_kernel (depthwise bias + 9 taps in order, fp16-
//        split MFMA over ascending channel quads, bias, residual, ReLU), so the outputs are
//        bit-identical to the per-op path; the next op's weights are loaded into registers while
//        this op computes and written to LDS after its barrier (two barriers per op).
//   round 6: NC is a template parameter of the task (a runtime NC made every MFMA triple
//        conditional: an accumulator copy and an MFMA drain per K-step), the K loop keeps the next
//        K-step's reads in flight while the current one computes, the first op (s2 from the
//        32x32 map in HBM) stages its source through LDS in two row bands (BFV_BAND) instead of
//        nine dependent global tap reads per K-step (22 % of the stage's cycles), and a tap map
//        leaves LDS by a coalesced 16-B copy during the next op (was 4-B stores in the epilogue).
// ------------------------------------------------------------------------------------------------
#define BFS_NW 8
#define BFS_PF 6     // float4 of the next op's W^T + dw table per thread (checked on the host)
#define BFS_BQ 16    // float4 of a staged band per thread (checked on the host)
#define BFV_GLOBAL 0  // first op, taps read from the map in global memory
#define BFV_BAND 1    // first op, s2 on a 16-wide output: source rows staged in LDS, two bands
#define BFV_DPP16 2   // s1 block on a 16-wide resident map (x-neighbour taps by DPP, no tap masks)
#define BFV_DPP8 3    // s1 block on an 8-wide resident map (x-neighbour taps by DPP)
#define BFV_S1 4      // s1 block on the resident map, nine tap reads
#define BFV_MP 5      // s2 max-pool block on the resident map
#define BFV_HEAD 6    // 1x1 detector head on the resident tap
// resident maps carry a zero row above and below (the map's row 0 sits one row into the map
// region, channel stride coutp + 4 of the op that wrote it): taps on rows -1 / H read zeros, the
// value the tap mask would give (bit-identical), so those taps need no mask

__device__ __forceinline__ int rfl(int v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ void bfs_wload(const BfSub& o, const float* P_, f32x4 (&pf)[BFS_PF]) {
  const int kq = o.cinp >> 2, nW = o.coutp * kq, nT = nW + (o.dw ? 10 * kq : 0);
#pragma unroll
  for (int i = 0; i < BFS_PF; ++i) {
    const int e = threadIdx.x + i * (BFS_NW * 64);
    const int n = e / kq, q = e - n * kq;
    const int off = e < nW ? o.pww + n * o.cinp + 4 * q : (e < nT ? o.dww + 4 * (e - nW) : 0);
    pf[i] = ld4(P_ + off);
  }
}

__device__ __forceinline__ void bfs_wstore(const BfSub& o, const f32x4 (&pf)[BFS_PF], float* wt, float* dwt) {
  const int kq = o.cinp >> 2, nW = o.coutp * kq, nT = nW + (o.dw ? 10 * kq : 0);
  wt += o.wto;
#pragma unroll
  for (int i = 0; i < BFS_PF; ++i) {
    const int e = threadIdx.x + i * (BFS_NW * 64);
    const int n = e / kq, q = e - n * kq;
    if (e < nW) *(f32x4*)(wt + n * o.ks + 4 * q) = split_w(pf[i]);
    else if (e < nT) *(f32x4*)(dwt + 4 * (e - nW)) = pf[i];
  }
}

// DPP (stride-1 depthwise ops on 16- or 8-wide maps from the LDS map): per 3x3 row one ds_read_b128
// of the centre column, the x-neighbours by DPP row shifts of it (a 16-lane DPP row is one 16-wide
// map row or two 8-wide ones; lanes whose neighbour is across a map-row edge are zeroed by the tap
// mask as before): 3 tap reads per K-step instead of 9, the same FMAs in the same order (bit-identical)
__device__ __forceinline__ float dpp_from_prev(float v) {  // lane i <- lane i - 1 of its 16-lane row
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x111, 0xf, 0xf, true));
}
__device__ __forceinline__ float dpp_from_next(float v) {  // lane i <- lane i + 1 of its 16-lane row
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x101, 0xf, 0xf, true));
}

#define BFS_MAXNC 3  // output-channel chunks per wave task (acc registers: 16 each)
#ifndef BFS_PIPE
#define BFS_PIPE 0   // 1: the K loop prefetches the next step's taps / W^T (more VGPRs: spills)
#endif
#ifndef BFS_PIPE1
#define BFS_PIPE1 0  // 1: the same for the single-chunk (NC = 1) tasks only (8x8 ops, heads): neutral
#endif
#ifdef BFS_SB_ON   // a scheduling barrier after each step's reads (measured slower: more spills)
#define BFS_SB() __builtin_amdgcn_sched_barrier(0)
#else
#define BFS_SB() do {} while (0)
#endif
// the streamed maps (the stage's source rows and the taps, each touched once) bypass L2 retention
// (non-temporal), so the stage's weights, re-read by every frame, stay L2-resident
#ifndef BFS_NT
#define BFS_NT 1
#endif
__device__ __forceinline__ f32x4 ld4_nt(const float* p) {
  if (BFS_NT) return __builtin_nontemporal_load((const f32x4*)p);
  return *(const f32x4*)p;
}
__device__ __forceinline__ void st4_nt(float* p, f32x4 v) {
  if (BFS_NT) __builtin_nontemporal_store(v, (f32x4*)p);
  else *(f32x4*)p = v;
}


// the prefetched reads of one K-step (8 input channels; this lane's quad c0 = 4 half + 8 k); the
// depthwise table rows (10 broadcast quads) are read inside the step, ahead of the taps' DPP work
template <int NT, int NC>
struct BfsK {
  f32x4 x[NT];                  // source taps (DPP: the 3 centre-column reads)
  f32x4 w[NC];                  // W^T quads (fp16 hi/lo pairs) of the NC output-channel chunks
};

// one wave task of op o: acc[j] (j < NC) = the final outputs (bias, residual, ReLU applied) of
// output-channel chunk grp * NC + j at the 32 positions of chunk `chunk`.  src: the source map
// (global: the stage input of this image; LDS: the resident map or, BFV_BAND, the staged rows
// iyb.. of the source), channel stride ss.
template <int V, int RES, int NC>
__device__ __forceinline__ void bfs_task(const BfSub& o, const float* src, int ss, int iyb, const float* wt,
                                         const float* dwt, const float* P_, int chunk, int grp,
                                         f32x16 (&acc)[BFS_MAXNC]) {
  constexpr bool DW = V != BFV_HEAD, DPP = V == BFV_DPP16 || V == BFV_DPP8;
  constexpr int NT = !DW ? 1 : (DPP ? 3 : 9), ND = DW ? 10 : 0;
  // taps that need the mask: rows -1 / H of a resident map are its zero halo rows; a 16-wide
  // map's x-neighbours come from DPP row shifts, zero at the row ends (bound_ctrl)
  constexpr bool YH = V == BFV_DPP16 || V == BFV_DPP8 || V == BFV_S1 || V == BFV_MP;
  auto masked = [](int tp) constexpr {
    const int dy = tp / 3, dx = tp % 3;
    if (V == BFV_DPP16) return false;
    if (V == BFV_MP) return dx == 2;
    if (YH) return dx != 1;
    (void)dy;
    return true;
  };
  const int lane = threadIdx.x & 63, half = lane >> 5, l32 = lane & 31;
  // the op's fields as wave-uniform registers (left as references the compiler re-loads them
  // from kernarg inside the K loop, each s_load behind an lgkmcnt(0))
  const int cinp = rfl(o.cinp), ks = rfl(o.ks), coutp = rfl(o.coutp);
  const int ow = rfl(o.w), wo = rfl(o.wo), oh = rfl(o.h), S = rfl(o.s), padt = rfl(o.padt), padl = rfl(o.padl);
  const int lgWo = __builtin_ctz(wo);
  const int p = chunk * 32 + l32;
  const int oy = p >> lgWo, ox = p & (wo - 1);
  int toff[9];
  uint32_t tmask = 0;
  {
    // masked taps read the centre tap's (always valid) offset: no read outside the staged rows
    const int cy = oy * S - padt + 1, cx = ox * S - padl + 1;
    const bool cok = cy >= 0 && cy < oh && cx >= 0 && cx < ow;
    const int cen = cok ? ((cy - iyb) * ow + cx) * ss : 0;
#pragma unroll
    for (int tp = 0; tp < 9; ++tp) {
      const int iy = oy * S - padt + tp / 3, ix = ox * S - padl + tp % 3;
      const bool ok = iy >= 0 && iy < oh && ix >= 0 && ix < ow;
      // an unmasked tap's row may be a halo row (x always in range for those)
      toff[tp] = ok || !masked(tp) ? ((iy - iyb) * ow + ix) * ss : cen;
      tmask |= ok ? (1u << tp) : 0u;
    }
    if (!DW) toff[0] = ((oy - iyb) * ow + ox) * ss;
  }
  const int n0 = grp * NC * 32 + l32;
  float bias[NC];
  int wrow[NC];
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    const int n = n0 + 32 * j;
    bias[j] = n < coutp ? P_[o.pwb + n] : 0.f;
    wrow[j] = (n < coutp ? n : coutp - 1) * ks;  // columns past coutp: finite weights, outputs unused
  }
#pragma unroll
  for (int j = 0; j < NC; ++j) acc[j] = (f32x16){};

  using K = BfsK<NT, NC>;
  typedef f32x4 Dv[ND > 0 ? ND : 1];
  auto load = [&](int c0, K& r) {
#pragma unroll
    for (int t = 0; t < NT; ++t) r.x[t] = ld4(src + toff[DPP ? 3 * t + 1 : t] + c0);
#pragma unroll
    for (int j = 0; j < NC; ++j) r.w[j] = ld4(wt + wrow[j] + c0);
  };
  // the step's depthwise table rows, issued as one batch ahead of the prefetch of the next step
  // (left to the scheduler, each row was read behind its own lgkmcnt(0): an LDS round trip per row)
  auto load_dw = [&](int c0, Dv& dv) {
#pragma unroll
    for (int t = 0; t < ND; ++t) dv[t] = ld4(dwt + t * cinp + c0);
  };
  auto step = [&](const K& r, const Dv& dv) {
    f32x4 av;
    if constexpr (DW) {
      f32x4 xv[9];
      if constexpr (DPP) {
#pragma unroll
        for (int dy = 0; dy < 3; ++dy) {
          const f32x4 c = r.x[dy];
          xv[3 * dy + 1] = c;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            xv[3 * dy][e] = dpp_from_prev(c[e]);
            xv[3 * dy + 2][e] = dpp_from_next(c[e]);
          }
        }
      } else {
#pragma unroll
        for (int tp = 0; tp < 9; ++tp) xv[tp] = r.x[tp];
      }
      av = dv[9];
#pragma unroll
      for (int tp = 0; tp < 9; ++tp) {
        const f32x4 x = !masked(tp) || ((tmask >> tp) & 1u) ? xv[tp] : f32x4{0.f, 0.f, 0.f, 0.f};
        const f32x4 wv = dv[tp];
        av.x = fmaf(x.x, wv.x, av.x);
        av.y = fmaf(x.y, wv.y, av.y);
        av.z = fmaf(x.z, wv.z, av.z);
        av.w = fmaf(x.w, wv.w, av.w);
      }
    } else {
      av = r.x[0];
    }
#pragma unroll
    for (int j = 0; j < NC; ++j) acc[j] = mfma_split(av, r.w[j], acc[j]);
  };
  // K loop, two steps per trip: the next step's reads are issued before this step's arithmetic
  // (BFV_BAND: one buffer, its registers hold the second band's staged rows meanwhile; BFV_GLOBAL
  // too, the generic fallback)
  const int nks = cinp >> 3;
  int c0 = 4 * half;
  Dv dv;
  if constexpr (V == BFV_BAND || V == BFV_GLOBAL || !(BFS_PIPE || (BFS_PIPE1 && NC == 1))) {
    for (int k = 0; k < nks; ++k, c0 += 8) {
      K A;
      load_dw(c0, dv);
      load(c0, A);
      if constexpr (V != BFV_BAND && V != BFV_GLOBAL) BFS_SB();
      step(A, dv);
    }
  } else {
    K A, B;
    load(c0, A);
    int k = 0;
    for (; k + 2 <= nks; k += 2, c0 += 16) {
      load_dw(c0, dv);
      load(c0 + 8, B);
      BFS_SB();
      step(A, dv);
      load_dw(c0 + 8, dv);
      load(k + 2 < nks ? c0 + 16 : c0 + 8, A);
      BFS_SB();
      step(B, dv);
    }
    if (nks & 1) {
      load_dw(c0, dv);
      BFS_SB();
      step(A, dv);
    }
  }

  // epilogue values: lane = output channel n, registers = 16 positions of the chunk
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    const int n = n0 + 32 * j;
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const int q = chunk * 32 + (g & 3) + 8 * (g >> 2) + 4 * half;
      const int qy = q >> lgWo, qx = q & (wo - 1);
      float v = acc[j][g] + bias[j];
      if (RES == BF_RES_ID) {
        if (n < cinp) v += src[((qy - iyb) * ow + qx) * ss + n];
      } else if (RES == BF_RES_MAXPOOL) {
        if (n < cinp) {
          const float* t = src + ((2 * qy - iyb) * ow + 2 * qx) * ss + n;
          v += fmaxf(fmaxf(t[0], t[ss]), fmaxf(t[ow * ss], t[ow * ss + ss]));
        }
      }
      if (DW) v = v > 0.f ? v : 0.f;
      acc[j][g] = v;
    }
  }
}

// the task of op o for this wave (variant and NC dispatched to the compile-time instantiations)
__device__ __forceinline__ void bfs_dispatch(const BfSub& o, int var, int nc, const float* src, int ss, int iyb,
                                             const float* wt, const float* dwt, const float* P_, int chunk,
                                             int grp, f32x16 (&acc)[BFS_MAXNC]) {
  const int res = rfl(o.res);
#define BFS_NCS(V_, R_)                                                              \
  switch (nc) {                                                                      \
    case 1: bfs_task<V_, R_, 1>(o, src, ss, iyb, wt, dwt, P_, chunk, grp, acc); break; \
    case 2: bfs_task<V_, R_, 2>(o, src, ss, iyb, wt, dwt, P_, chunk, grp, acc); break; \
    default: bfs_task<V_, R_, 3>(o, src, ss, iyb, wt, dwt, P_, chunk, grp, acc); break; \
  }
  switch (var) {
    case BFV_GLOBAL:
      if (res == BF_RES_MAXPOOL) { BFS_NCS(BFV_GLOBAL, BF_RES_MAXPOOL) } else { BFS_NCS(BFV_GLOBAL, BF_RES_ID) }
      break;
    case BFV_BAND: bfs_task<BFV_BAND, BF_RES_MAXPOOL, 1>(o, src, ss, iyb, wt, dwt, P_, chunk, grp, acc); break;
    case BFV_DPP16: BFS_NCS(BFV_DPP16, BF_RES_ID) break;
    case BFV_DPP8: BFS_NCS(BFV_DPP8, BF_RES_ID) break;
    case BFV_S1: BFS_NCS(BFV_S1, BF_RES_ID) break;
    case BFV_MP: BFS_NCS(BFV_MP, BF_RES_MAXPOOL) break;
    default: BFS_NCS(BFV_HEAD, BF_RES_NONE) break;
  }
#undef BFS_NCS
}

// BFV_BAND staging: rows [r0, r1) of the source map (contiguous in global memory) into LDS at
// channel stride sst; registers first (the second band's loads fly during the first band's work)
__device__ __forceinline__ void bfs_band_load(const float* g, int nq, f32x4 (&r)[BFS_BQ]) {
#pragma unroll
  for (int i = 0; i < BFS_BQ; ++i) {
    const int e = threadIdx.x + i * (BFS_NW * 64);
    r[i] = ld4_nt(g + 4 * (e < nq ? e : nq - 1));
  }
}
__device__ __forceinline__ void bfs_band_store(float* st, int nq, int kq, int sst, const f32x4 (&r)[BFS_BQ]) {
  const float inv = 1.f / (float)kq;
#pragma unroll
  for (int i = 0; i < BFS_BQ; ++i) {
    const int e = threadIdx.x + i * (BFS_NW * 64);
    if (e < nq) {
      const int pix = (int)(((float)e + 0.5f) * inv), q = e - pix * kq;  // exact for e < 2^16
      *(f32x4*)(st + pix * sst + 4 * q) = r[i];
    }
  }
}

// the epilogue stores of one wave task: the map (blocks) and / or the head outputs in HBM
__device__ __forceinline__ void bfs_store(const BfSub& o, const float* const* bufs, float* map, int cs, int64_t img,
                                          int chunk, int grp, const f32x16 (&acc)[BFS_MAXNC]) {  // map: row 0
  const int lane = threadIdx.x & 63, half = lane >> 5, l32 = lane & 31;
  const int64_t hwo = o.ho * o.wo;
  const bool head = !o.dw;
  float* gd = head ? (float*)bufs[o.gdst] : nullptr;
  float* gd2 = head && o.split ? (float*)bufs[o.gdst2] : nullptr;
  const int nc = rfl(o.nc), coutp = rfl(o.coutp);
  const int split = rfl(o.split), cout = rfl(o.cout), ostride = rfl(o.ostride);
#pragma unroll
  for (int j = 0; j < BFS_MAXNC; ++j) {
    if (j >= nc) continue;
    const int n = (grp * nc + j) * 32 + l32;
    if (n >= coutp) continue;
    if (!head) {
#pragma unroll
      for (int g = 0; g < 16; ++g) map[(chunk * 32 + (g & 3) + 8 * (g >> 2) + 4 * half) * cs + n] = acc[j][g];
      continue;
    }
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const int q = chunk * 32 + (g & 3) + 8 * (g >> 2) + 4 * half;
      const float v = acc[j][g];
      const int64_t pos = img * hwo + q;
      // plain stores: 4-B non-temporal stores of these scattered head outputs reach HBM as partial
      // lines (the stage's PMC write bytes 216 MB with them, 190 MB without)
      if (split) {
        if (n < split) gd[pos * split + n] = v;
        else if (n < cout) gd2[pos * (cout - split) + (n - split)] = v;
      } else if (n < ostride) {
        gd[pos * ostride + n] = v;
      }
    }
  }
}

// a tap map (the resident map after op o) to its caller buffer: [img][HW][coutp], 16-B pieces
__device__ __forceinline__ void bfs_tap_copy(const BfSub& o, const float* const* bufs, const float* lmap, int64_t img) {
  const int kq = rfl(o.coutp) >> 2, hw = rfl(o.ho * o.wo), nq = hw * kq, cs = rfl(o.cso);
  const float* map = lmap + rfl(o.wo) * cs;  // row 0
  float* gd = (float*)bufs[o.gdst] + img * hw * (kq * 4);
  const float inv = 1.f / (float)kq;
  for (int e = threadIdx.x; e < nq; e += BFS_NW * 64) {
    const int pix = (int)(((float)e + 0.5f) * inv), q = e - pix * kq;
    st4_nt(gd + 4 * e, ld4(map + pix * cs + 4 * q));
  }
}

__global__ void __launch_bounds__(BFS_NW * 64) bf_stage_kernel(BfStageArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* map = lds;
  float* wt = lds + a.map_floats;
  float* dwt = wt + a.wt_floats;
  const int64_t img = blockIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const float* P_ = a.params;
  f32x4 pf[BFS_PF];
  bfs_wload(a.op[0], P_, pf);
  bfs_wstore(a.op[0], pf, wt, dwt);
  __syncthreads();
#ifdef BFS_STAMPS   // per-op, per-wave cycles of workgroup 0: compute | barrier 1 | stores | barrier 2
  uint32_t bst[BFS_MAX][4];
  uint64_t bt = __builtin_amdgcn_s_memtime();
#define BFS_ST(i, k) do { const uint64_t t_ = __builtin_amdgcn_s_memtime(); bst[i][k] = (uint32_t)(t_ - bt); bt = t_; } while (0)
#else
#define BFS_ST(i, k) do {} while (0)
#endif
  int tap = -1;  // op whose output map is a tap still to be copied out of LDS
  for (int i = 0; i < a.nops; ++i) {
    const BfSub& o = a.op[i];
    if (i + 1 < a.nops) bfs_wload(a.op[i + 1], P_, pf);
    if (tap >= 0) bfs_tap_copy(a.op[tap], a.bufs, map, img);  // the map is rewritten after barrier 1
    tap = -1;
    const int var = rfl(o.var), nc = rfl(o.nc);
    const int ngrp = rfl(o.nct) / nc;
    const float* wto = wt + rfl(o.wto);
    f32x16 acc[BFS_MAXNC], acc2[BFS_MAXNC];
    int chunk, chunk2 = -1, grp;
    if (var == BFV_BAND) {
      // two bands of output rows, each 4 chunks x ngrp tasks; the source rows of band b:
      // [b H / 2, b H / 2 + H / 2 + 1) clipped to the map, staged at LDS offset 0 (stride sst)
      const int H = rfl(o.h), W = rfl(o.w), kq = rfl(o.cinp) >> 2, sst = rfl(o.sst);
      const float* gsrc = a.src + img * H * W * (kq * 4);
      const int hb = H >> 1;
      const int nq0 = (hb + 1) * W * kq, nq1 = (H - hb) * W * kq;
      f32x4 r[BFS_BQ];
      bfs_band_load(gsrc, nq0, r);
      bfs_band_store(lds, nq0, kq, sst, r);
      bfs_band_load(gsrc + hb * W * kq * 4, nq1, r);  // in flight over band 0
      __syncthreads();
      const bool busy = wave < 4 * ngrp;
      chunk = busy ? wave / ngrp : -1;
      grp = wave - (wave / ngrp) * ngrp;
      if (busy) bfs_dispatch(o, var, nc, lds, sst, 0, wto, dwt, P_, chunk, grp, acc);
      __syncthreads();
      bfs_band_store(lds, nq1, kq, sst, r);
      __syncthreads();
      chunk2 = busy ? chunk + 4 : -1;
      if (busy) bfs_dispatch(o, var, nc, lds, sst, hb, wto, dwt, P_, chunk2, grp, acc2);
    } else {
      const int ntask = ((rfl(o.ho) * rfl(o.wo)) >> 5) * ngrp;
      chunk = wave / ngrp;
      grp = wave - chunk * ngrp;
      if (wave < ntask) {
        if (var == BFV_GLOBAL) {
          const float* gs = a.src + img * o.h * o.w * o.cinp;
          bfs_dispatch(o, var, nc, gs, rfl(o.cinp), 0, wto, dwt, P_, chunk, grp, acc);
        } else {
          const int ss = rfl(o.ss);
          bfs_dispatch(o, var, nc, map + rfl(o.w) * ss, ss, 0, wto, dwt, P_, chunk, grp, acc);
        }
      } else {
        chunk = -1;
      }
    }
    BFS_ST(i, 0);
    __syncthreads();  // every wave's reads of the map and of W^T are done
    BFS_ST(i, 1);
    {
      const int cso = rfl(o.cso), wo = rfl(o.wo);
      float* orow = map + wo * cso;
      if (chunk >= 0) bfs_store(o, a.bufs, orow, cso, img, chunk, grp, acc);
      if (chunk2 >= 0) bfs_store(o, a.bufs, orow, cso, img, chunk2, grp, acc2);
      if (o.zhalo) {  // rows -1 and HO of the new map
        const int rq = wo * cso / 4, ho = rfl(o.ho);
        for (int e = threadIdx.x; e < 2 * rq; e += BFS_NW * 64)
          *(f32x4*)(map + (e < rq ? 4 * e : (ho + 1) * wo * cso + 4 * (e - rq))) = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    if (o.dw && o.gdst >= 0) tap = i;
    if (i + 1 < a.nops) bfs_wstore(a.op[i + 1], pf, wt, dwt);
    BFS_ST(i, 2);
    __syncthreads();  // outputs and the next op's weights visible
    BFS_ST(i, 3);
  }
  if (tap >= 0) bfs_tap_copy(a.op[tap], a.bufs, map, img);
#ifdef BFS_STAMPS
  if (blockIdx.x == 0 && (threadIdx.x & 63) == 0)
    for (int i = 0; i < a.nops; ++i)
      printf("BFS op %d w %d comp %u bar1 %u store %u bar2 %u\n", i, wave, bst[i][0], bst[i][1], bst[i][2], bst[i][3]);
#endif
#undef BFS_ST
}

typedef void (*bf_fn)(BfArgs);

// compile-time channel specialisations of the BlazeFace 64x64 / 32x32 stages (CS = KS = CINP + 4,
// output stride COUTP, all output-channel chunks in one task); anything else runs the generic one
static bf_fn pick_rows(int s, int nc, int cinp = 0, int coutp = 0, int cs = 0, int ks = 0, int ostride = 0, int nct = 0) {
  if (cs == cinp + 4 && ks == cinp + 4 && ostride == coutp && nct == (coutp + 31) / 32 && nc == nct) {
#define BF_ROWS_T(S_, CI_, CO_) if (s == S_ && cinp == CI_ && coutp == CO_) return bf_rows_kernel<S_, 0, CI_, CO_>;
    BF_ROWS_T(1, 24, 24)
    BF_ROWS_T(1, 24, 32)
    BF_ROWS_T(2, 32, 32)
    BF_ROWS_T(1, 32, 40)
    BF_ROWS_T(1, 40, 48)
    BF_ROWS_T(2, 48, 48)
#undef BF_ROWS_T
  }
  if (s == 1 && nc == 1) return bf_rows_kernel<1, 1, 0, 0>;
  if (s == 1 && nc == 2) return bf_rows_kernel<1, 2, 0, 0>;
  if (s == 2 && nc == 1) return bf_rows_kernel<2, 1, 0, 0>;
  if (s == 2 && nc == 2) return bf_rows_kernel<2, 2, 0, 0>;
  return nullptr;
}
static bf_fn pick_rows_op(const int* f) {
  return pick_rows(f[BFO_STRIDE], f[BFO_NC], f[BFO_CINP], f[BFO_COUTP], f[BFO_CS], f[BFO_KS], f[BFO_OSTRIDE], f[BFO_NCT]);
}

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

static bf_fn pick_direct(int s, int dw, int nc) {
#define BF_DNC(S_, DW_)                                  \
  switch (nc) {                                          \
    case 1: return bf_direct_kernel<S_, DW_, 1>;         \
    case 2: return bf_direct_kernel<S_, DW_, 2>;         \
    case 3: return bf_direct_kernel<S_, DW_, 3>;         \
    case 4: return bf_direct_kernel<S_, DW_, 4>;         \
    default: return nullptr;                             \
  }
  if (s == 1 && dw) { BF_DNC(1, 1) }
  if (s == 2 && dw) { BF_DNC(2, 1) }
  if (s == 1 && !dw) { BF_DNC(1, 0) }
#undef BF_DNC
  return nullptr;
}

// ------------------------------------------------------------------------------------------------
// front: the stem and the five blocks on the 64x64 / 32x32 maps (every layer before the stage) as
// ONE launch, one 8-wave workgroup per frame (persistent over frames).  The per-op kernels write
// every intermediate map to HBM and read it back (3.2 MB per frame, 58 % of the forward's time at
// 1,024 frames); here the maps stream row by row through LDS rings — each layer's output rows
// land in the next layer's input ring (4 rows: the 3 its 3x3 window reads + the one being
// written) — and only the frame (196 KB) and the last block's 32x32x48 output (196 KB) touch HBM.
//   * wave roles (fixed; waves w and w + 4 share a SIMD): w0/w1 the stem's two 32-position chunks of
//     a 64-wide row, w2/w3 block 1, w4/w5 block 2, w6 block 3 (odd phases, s2 32-wide) and the
//     frame's input rows (LDS-DMA two phases ahead into a 10-row ring: a phase waits only for the
//     pieces issued in the phase before it, not for its own), w7 block 4 (even) and block 5 (odd,
//     its rows to HBM).  The
//     pointwise weights of a wave's layers live in its registers (fp16 hi/lo pairs), the depthwise
//     tables in LDS.
//   * phase p (one workgroup barrier each, 76 per frame): stem row p, block-1 row p - 2, block-2
//     row p - 4, block-3 row (p - 7) / 2, block-4 row (p - 10) / 2, block-5 row (p - 13) / 2 —
//     every row a layer reads was written in an earlier phase, and the ring slot a layer writes
//     (row mod 4) is one no layer reads in that phase.  The bottom padding row of each map is
//     written as zeros by its producer, the top one and the column halos are the per-frame zeroing.
//   * the same arithmetic as bf_stem_kernel / bf_rows_kernel (stem: fp16-split MFMA over the same K
//     order and scales; blocks: depthwise bias + 9 taps in order, mfma_split per 8 channels in the
//     same order, bias + residual + ReLU): the output is bit-identical to the per-op launches.
// The geometry is the BlazeFace backbone's (host-checked against the plan records).
// ------------------------------------------------------------------------------------------------
#define BFF_NW 8
#ifndef BFF_SPLIT45
#define BFF_SPLIT45 1   // w2 both block-1 chunks; w3 and w7 one output-channel chunk each of blocks 4 / 5
#endif
#ifdef BFF_STAMPS   // per-wave busy cycles (task time, barrier waits excluded) of workgroup 0
#define BFF_BAR() do { bff_busy += __builtin_amdgcn_s_memtime() - bff_t0; bar_lds(); bff_t0 = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define BFF_BAR() bar_lds()
#endif
#define BFF_PHASES 76
#define BFF_INS 396        // floats per input-row slot: [4 zero][128 x 3][8 zero] (16-B aligned rows)
template <int K> struct BffL;  // block K (1..5): input map geometry of its LDS ring
//                                S  CINP COUTP  CS  COLS PADT PADL  WO  HO  ring offset (floats)
template <> struct BffL<1> { static constexpr int S = 1, CINP = 24, COUTP = 24, CS = 28, COLS = 66, PADT = 1, PADL = 1, WO = 64, HO = 64, RING = 0; };
template <> struct BffL<2> { static constexpr int S = 1, CINP = 24, COUTP = 32, CS = 28, COLS = 66, PADT = 1, PADL = 1, WO = 64, HO = 64, RING = 7392; };
template <> struct BffL<3> { static constexpr int S = 2, CINP = 32, COUTP = 32, CS = 36, COLS = 65, PADT = 0, PADL = 0, WO = 32, HO = 32, RING = 14784; };
template <> struct BffL<4> { static constexpr int S = 1, CINP = 32, COUTP = 40, CS = 36, COLS = 34, PADT = 1, PADL = 1, WO = 32, HO = 32, RING = 24144; };
template <> struct BffL<5> { static constexpr int S = 1, CINP = 40, COUTP = 48, CS = 44, COLS = 34, PADT = 1, PADL = 1, WO = 32, HO = 32, RING = 29040; };
#define BFF_RINGS 35024    // floats of the five rings (4 rows each)
#define BFF_NIN 10         // input ring rows: 6 read per phase + 2 landing + 2 in flight
#define BFF_IN BFF_RINGS   // input ring: BFF_NIN rows of BFF_INS
#define BFF_DW (BFF_IN + BFF_NIN * BFF_INS)
#define BFF_DWOFF(K) (BFF_DW + ((K) > 1 ? 240 : 0) + ((K) > 2 ? 240 : 0) + ((K) > 3 ? 320 : 0) + ((K) > 4 ? 320 : 0))
#define BFF_FLOATS (BFF_DW + 1520)
static_assert(BffL<5>::RING + 4 * BffL<5>::COLS * BffL<5>::CS == BFF_RINGS, "front rings");
static_assert(4 * BFF_FLOATS <= 160 * 1024, "front LDS");

struct BfFrontArgs {
  int stem[BFO_WORDS];
  int dww[6], pww[6], pwb[6];  // parameter offsets of blocks 1..5
  const float* params;
  const float* src;   // frames [n][128][128][3]
  float* dst;         // block 5's output [n][32][32][48]
  int64_t nimg;
};

// pointwise weights of block K for this lane (output channel nc * 32 + l32, channel quads
// c0 = 4 half + 8 k): the split_w pairs bf_rows_kernel keeps in LDS
// (output-channel chunks NC0 .. NC0 + NCN - 1)
template <int K, int NC0 = 0, int NCN = (BffL<K>::COUTP + 31) / 32>
__device__ __forceinline__ void bff_wload(const BfFrontArgs& a, f32x4 (&wr)[NCN][BffL<K>::CINP / 8],
                                          float (&bias)[NCN], int l32, int half) {
  using L = BffL<K>;
  constexpr int NKS = L::CINP / 8;
#pragma unroll
  for (int nc = 0; nc < NCN; ++nc) {
    const int n = (NC0 + nc) * 32 + l32;
#pragma unroll
    for (int k = 0; k < NKS; ++k)
      wr[nc][k] = n < L::COUTP ? split_w(ld4(a.params + a.pww[K] + n * L::CINP + 4 * half + 8 * k)) : f32x4{0.f, 0.f, 0.f, 0.f};
    bias[nc] = n < L::COUTP ? a.params[a.pwb[K] + n] : 0.f;
  }
}

// one 32-position chunk (c) of output row oy of block K: bf_rows_kernel's compute + epilogue; the
// output goes to block K + 1's ring (row slot oy & 3) or, for K = 5, to HBM; zero: the bottom
// padding row (zeros)
template <int K>
__device__ __forceinline__ void bff_dwload(const BfFrontArgs& a, f32x4 (&dwr)[BffL<K>::CINP / 8][10], int half) {
#pragma unroll
  for (int k = 0; k < BffL<K>::CINP / 8; ++k)
#pragma unroll
    for (int t = 0; t < 10; ++t) dwr[k][t] = ld4(a.params + a.dww[K] + t * BffL<K>::CINP + 4 * half + 8 * k);
}

// DWR: the depthwise table of the lane's channel quads in registers (dwr, bff_dwload) instead of
// 10 ds_read_b128 per K-step from the LDS copy (the front is LDS-bandwidth-bound).  NC0 / NC: the
// output-channel chunks this wave computes (two waves may share a row, each with its own chunks:
// the same depthwise, each chunk's products in the same order)
template <int K, bool DWR = false, int NC0 = 0, int NC = (BffL<K>::COUTP + 31) / 32>
__device__ __forceinline__ void bff_block(float* lds, int oy, int c, bool zero,
                                          const f32x4 (&wr)[NC][BffL<K>::CINP / 8],
                                          const float (&bias)[NC], float* gout, int l32, int half,
                                          const f32x4 (*dwr)[10] = nullptr) {
  using L = BffL<K>;
  constexpr int NKS = L::CINP / 8, ROW = L::COLS * L::CS;
  f32x16 acc[NC];
#pragma unroll
  for (int nc = 0; nc < NC; ++nc) acc[nc] = (f32x16){};
  const float* ring = lds + L::RING;
  const int iy0 = oy * L::S - L::PADT;
  if (!zero) {
    const int colx = (32 * c + l32) * L::S * L::CS;
    const float* r0 = ring + ((iy0 + 4) & 3) * ROW + colx;
    const float* r1 = ring + ((iy0 + 5) & 3) * ROW + colx;
    const float* r2 = ring + ((iy0 + 6) & 3) * ROW + colx;
    const float* dwt = lds + BFF_DWOFF(K);
#pragma unroll
    for (int k = 0; k < NKS; ++k) {
      const int c0 = 4 * half + 8 * k;
      f32x4 av = DWR ? dwr[k][9] : ld4(dwt + 9 * L::CINP + c0);
#pragma unroll
      for (int tp = 0; tp < 9; ++tp) {
        const float* rp = tp < 3 ? r0 : (tp < 6 ? r1 : r2);
        const f32x4 xv = ld4(rp + (tp % 3) * L::CS + c0);
        const f32x4 wv = DWR ? dwr[k][tp] : ld4(dwt + tp * L::CINP + c0);
        av.x = fmaf(xv.x, wv.x, av.x);
        av.y = fmaf(xv.y, wv.y, av.y);
        av.z = fmaf(xv.z, wv.z, av.z);
        av.w = fmaf(xv.w, wv.w, av.w);
      }
#pragma unroll
      for (int nc = 0; nc < NC; ++nc) acc[nc] = mfma_split(av, wr[nc][k], acc[nc]);
    }
  }
  // epilogue: lane = output channel, register g = position 32 c + 4 half + (g & 3) + 8 (g >> 2).
  // Every residual read of the row is issued before the first output write: the writes go to the
  // next layer's ring in the same LDS array, which the compiler cannot tell apart from this ring, so
  // read-write-read-... interleaved put each read behind its own lgkmcnt(0) (an LDS round trip per
  // output register; round 6)
#ifndef BFF_RESB
#define BFF_RESB 1
#endif
  float res[NC][16];
  if (BFF_RESB && !zero) {
#pragma unroll
    for (int nc = 0; nc < NC; ++nc) {
      const int n = min((NC0 + nc) * 32 + l32, L::CINP - 1);  // n >= CINP: read a valid address, unused
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const int x = 32 * c + 4 * half + (g & 3) + 8 * (g >> 2);
        if (L::S == 1) {
          res[nc][g] = ring[(oy & 3) * ROW + (x + L::PADL) * L::CS + n];
        } else {
          const float* t0 = ring + ((2 * oy) & 3) * ROW + 2 * x * L::CS + n;
          const float* t1 = ring + ((2 * oy + 1) & 3) * ROW + 2 * x * L::CS + n;
          res[nc][g] = fmaxf(fmaxf(t0[0], t0[L::CS]), fmaxf(t1[0], t1[L::CS]));
        }
      }
    }
  }
#pragma unroll
  for (int nc = 0; nc < NC; ++nc) {
    const int n = (NC0 + nc) * 32 + l32;
    if (n >= L::COUTP) continue;
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const int x = 32 * c + 4 * half + (g & 3) + 8 * (g >> 2);
      float v = 0.f;
      if (!zero) {
        v = acc[nc][g] + bias[nc];
        if (n < L::CINP) {
          if (BFF_RESB) {
            v += res[nc][g];
          } else if (L::S == 1) {
            v += ring[(oy & 3) * ROW + (x + L::PADL) * L::CS + n];
          } else {
            const float* t0 = ring + ((2 * oy) & 3) * ROW + 2 * x * L::CS + n;
            const float* t1 = ring + ((2 * oy + 1) & 3) * ROW + 2 * x * L::CS + n;
            v += fmaxf(fmaxf(t0[0], t0[L::CS]), fmaxf(t1[0], t1[L::CS]));
          }
        }
        v = v > 0.f ? v : 0.f;
      }
      if constexpr (K < 5) {
        using O = BffL<K + 1>;
        lds[O::RING + (oy & 3) * (O::COLS * O::CS) + (x + O::PADL) * O::CS + n] = v;
      } else {
        gout[(oy * L::WO + x) * L::COUTP + n] = v;
      }
    }
  }
}

__global__ void __launch_bounds__(BFF_NW * 64) bf_front_kernel(BfFrontArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int lane = threadIdx.x & 63, half = lane >> 5, l32 = lane & 31;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const float* P_ = a.params;
#ifdef BFF_STAMPS
  uint64_t bff_busy = 0, bff_t0 = __builtin_amdgcn_s_memtime();
  const uint64_t bff_start = bff_t0;
#endif
  // depthwise tables of blocks 1..5 (10 x CINP each) and the input ring's zero pads, once per launch
  {
    const int cinp[6] = {0, 24, 24, 32, 32, 40};
    for (int k = 1; k <= 5; ++k)
      for (int i = threadIdx.x; i < 10 * cinp[k]; i += BFF_NW * 64) lds[BFF_DWOFF(k) + i] = P_[a.dww[k] + i];
    for (int i = threadIdx.x; i < BFF_NIN * BFF_INS / 4; i += BFF_NW * 64) *(f32x4*)(lds + BFF_IN + 4 * i) = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  __syncthreads();
  // per-frame prologue: zero the rings and the input slot of row -1; w6 lands input rows 0..6
  auto frame_begin = [&](int64_t img) {
    for (int i = threadIdx.x; i < BFF_RINGS / 4; i += BFF_NW * 64) *(f32x4*)(lds + 4 * i) = f32x4{0.f, 0.f, 0.f, 0.f};
    if (wave == 6) {
      for (int i = lane; i < BFF_INS / 4; i += 64) *(f32x4*)(lds + BFF_IN + (BFF_NIN - 1) * BFF_INS + 4 * i) = f32x4{0.f, 0.f, 0.f, 0.f};
      const float* fr = a.src + img * (128 * 128 * 3);
      for (int r = 0; r < 7; ++r) {
        glds16(fr + r * 384 + 4 * lane, lds_addr(lds + BFF_IN + r * BFF_INS + 4));
        if (lane < 32) glds16(fr + r * 384 + 256 + 4 * lane, lds_addr(lds + BFF_IN + r * BFF_INS + 4 + 256));
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
  };

  if (wave < 2) {
    // ---- stem (bf_stem_kernel's arithmetic): 32 positions ox = 32 wave + l32 of row p ----
    const int* f = a.stem;
    SplitW wsp[STEM_NK];
    float inv;
    {
      f32x8 v[STEM_NK];
      float mx = 0.f;
#pragma unroll
      for (int s = 0; s < STEM_NK; ++s) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int q = 8 * s + j;
          v[s][j] = q < STEM_KS ? P_[f[BFO_PWW] + l32 * 90 + half * STEM_KS + q] : 0.f;
          mx = fmaxf(mx, fabsf(v[s][j]));
        }
      }
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float s1 = pow2_scale(mx, 13);
      inv = SPLIT_INV_C / s1;
#pragma unroll
      for (int s = 0; s < STEM_NK; ++s) wsp[s] = split_w8(v[s] * s1);
    }
    const int cout = f[BFO_COUT];
    const float bias = l32 < cout ? P_[f[BFO_PWB] + l32] : 0.f;
    for (int64_t img = blockIdx.x; img < a.nimg; img += gridDim.x) {
      frame_begin(img);
      for (int p = 0; p < BFF_PHASES; ++p) {
        if (p <= 64) {
          f32x16 acc = {};
          if (p < 64) {
            const int ox = 32 * wave + l32;
            // input rows 2p - 1 + 3 half + k (k = ky - 3 half), slot = row mod BFF_NIN; element (ky, kx, c)
            // of the lane's 5x5 window at 1 + 6 ox + 3 kx + c within the slot (image column -1 in the pad)
            const float* tr[3];
#pragma unroll
            for (int k = 0; k < 3; ++k) tr[k] = lds + BFF_IN + ((2 * p - 1 + 3 * half + k + BFF_NIN) % BFF_NIN) * BFF_INS + 1 + 6 * ox;
#pragma unroll
            for (int s = 0; s < STEM_NK; ++s) {
              f32x8 xv;
#pragma unroll
              for (int j = 0; j < 8; ++j) {
                const int q = 8 * s + j;
                xv[j] = q < STEM_KS ? tr[q / 15][((q / 3) % 5) * 3 + q % 3] : 0.f;
              }
              acc = mfma3_dw(split_d8(xv), wsp[s], acc);
            }
          }
          if (l32 < cout) {
            using O = BffL<1>;
            float* drow = lds + O::RING + (p & 3) * (O::COLS * O::CS) + O::PADL * O::CS + l32;
#pragma unroll
            for (int g = 0; g < 16; ++g) {
              const int x = 32 * wave + 4 * half + (g & 3) + 8 * (g >> 2);
              float v = 0.f;
              if (p < 64) {
                v = fmaf(acc[g], inv, bias);
                v = v > 0.f ? v : 0.f;
              }
              drow[x * O::CS] = v;
            }
          }
        }
        BFF_BAR();
      }
    }
  } else if (wave == 2 || (wave == 3 && !BFF_SPLIT45)) {
    f32x4 wr[1][3], dwr[3][10];
    float bias[1];
    bff_wload<1>(a, wr, bias, l32, half);
    bff_dwload<1>(a, dwr, half);
    for (int64_t img = blockIdx.x; img < a.nimg; img += gridDim.x) {
      frame_begin(img);
      for (int p = 0; p < BFF_PHASES; ++p) {
        const int oy = p - 2;
        if (oy >= 0 && oy <= 64) {
          bff_block<1, true>(lds, oy, wave - 2, oy == 64, wr, bias, nullptr, l32, half, dwr);
          if (BFF_SPLIT45) bff_block<1, true>(lds, oy, 1, oy == 64, wr, bias, nullptr, l32, half, dwr);
        }
        BFF_BAR();
      }
    }
  } else if (wave == 3) {
    // blocks 4 / 5's second output-channel chunk (w7 has the first)
    f32x4 w4[1][4], w5[1][5];
    float b4[1], b5[1];
    bff_wload<4, 1, 1>(a, w4, b4, l32, half);
    bff_wload<5, 1, 1>(a, w5, b5, l32, half);
    for (int64_t img = blockIdx.x; img < a.nimg; img += gridDim.x) {
      frame_begin(img);
      float* gout = a.dst + img * (32 * 32 * 48);
      for (int p = 0; p < BFF_PHASES; ++p) {
        if (p & 1) {
          if (p >= 13) bff_block<5, false, 1, 1>(lds, (p - 13) >> 1, 0, false, w5, b5, gout, l32, half);
        } else {
          const int oy = (p - 10) >> 1;
          if (p >= 10 && oy <= 32) bff_block<4, false, 1, 1>(lds, oy, 0, oy == 32, w4, b4, nullptr, l32, half);
        }
        BFF_BAR();
      }
    }
  } else if (wave < 6) {
    f32x4 wr[1][3], dwr[3][10];
    float bias[1];
    bff_wload<2>(a, wr, bias, l32, half);
    bff_dwload<2>(a, dwr, half);
    for (int64_t img = blockIdx.x; img < a.nimg; img += gridDim.x) {
      frame_begin(img);
      for (int p = 0; p < BFF_PHASES; ++p) {
        const int oy = p - 4;
        if (oy >= 0 && oy <= 64) bff_block<2, true>(lds, oy, wave - 4, oy == 64, wr, bias, nullptr, l32, half, dwr);
        BFF_BAR();
      }
    }
  } else if (wave == 6) {
    f32x4 w3[1][4];
    float b3[1];
    bff_wload<3>(a, w3, b3, l32, half);
    for (int64_t img = blockIdx.x; img < a.nimg; img += gridDim.x) {
      frame_begin(img);
      const float* fr = a.src + img * (128 * 128 * 3);
      for (int p = 0; p < BFF_PHASES; ++p) {
        if (p & 1) {
          const int oy = (p - 7) >> 1;
          if (p >= 7 && oy <= 32) bff_block<3>(lds, oy, 0, oy == 32, w3, b3, nullptr, l32, half);
        }
        // the input rows phase p + 2 adds (2p + 7, 2p + 8): zeros past the frame, LDS-DMA pieces
        // otherwise; then wait for the pieces of phase p - 1 only (this phase's stay in flight)
        int nd = 0;
        if (p < 62) {
#pragma unroll
          for (int k = 0; k < 2; ++k) {   // zero rows first: no LDS write behind this phase's pieces
            const int r = 2 * p + 7 + k;
            if (r >= 128)
              for (int i = lane; i < 96; i += 64) *(f32x4*)(lds + BFF_IN + (r % BFF_NIN) * BFF_INS + 4 + 4 * i) = f32x4{0.f, 0.f, 0.f, 0.f};
          }
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            const int r = 2 * p + 7 + k;
            if (r < 128) {
              float* d = lds + BFF_IN + (r % BFF_NIN) * BFF_INS + 4;
              glds16(fr + r * 384 + 4 * lane, lds_addr(d));
              if (lane < 32) glds16(fr + r * 384 + 256 + 4 * lane, lds_addr(d + 256));
              nd += 2;
            }
          }
        }
        if (nd == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else if (nd == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        BFF_BAR();
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  } else {
    constexpr int N45 = BFF_SPLIT45 ? 1 : 2;
    f32x4 w4[N45][4], w5[N45][5];
    float b4[N45], b5[N45];
    bff_wload<4, 0, N45>(a, w4, b4, l32, half);
    bff_wload<5, 0, N45>(a, w5, b5, l32, half);
    for (int64_t img = blockIdx.x; img < a.nimg; img += gridDim.x) {
      frame_begin(img);
      float* gout = a.dst + img * (32 * 32 * 48);
      for (int p = 0; p < BFF_PHASES; ++p) {
        if (p & 1) {
          if (p >= 13) bff_block<5, false, 0, N45>(lds, (p - 13) >> 1, 0, false, w5, b5, gout, l32, half);
        } else {
          const int oy = (p - 10) >> 1;
          if (p >= 10 && oy <= 32) bff_block<4, false, 0, N45>(lds, oy, 0, oy == 32, w4, b4, nullptr, l32, half);
        }
        BFF_BAR();
      }
    }
  }
#ifdef BFF_STAMPS
  if (blockIdx.x == 0 && lane == 0)
    printf("BFF w%d busy %llu total %llu\n", wave, (unsigned long long)bff_busy,
           (unsigned long long)(__builtin_amdgcn_s_memtime() - bff_start));
#endif
}

struct hpe_blazeface {
  int* words;
  int n_words;
  int nops;
  int64_t act_floats;
  int n_cu;
};

// stage task split: the fewest output-channel chunks per wave task (most waves busy) that keeps
// every task of an op on its own wave (<= BFS_NW tasks: results stay in registers over the barrier)
static int bfs_nc(int nchunk, int nct) {
  for (int nc = 1; nc <= nct && nc <= BFS_MAXNC; ++nc)
    if (nct % nc == 0 && nchunk * (nct / nc) <= BFS_NW) return nc;
  return 0;
}
// the NC a stage op runs with: BFS_NCMAX prefers the most output-channel chunks per task (fewer
// tasks, the depthwise work done once per position chunk) over the most busy waves
static int bfs_nc_run(int nchunk, int nct) {
#ifdef BFS_NCMAX
  for (int nc = nct < BFS_MAXNC ? nct : BFS_MAXNC; nc >= 1; --nc)
    if (nct % nc == 0 && nchunk * (nct / nc) <= BFS_NW) return nc;
#endif
  return bfs_nc(nchunk, nct);
}

// the task variant of stage op k (record g); the band op (the first op, s2 onto a 16x16 map) also
// gets its W^T placed at the end of the W^T region (wto), clear of its staged source rows, which
// start at LDS offset 0 (stride sst), and its own NC (4 chunks per band)
static int bfs_variant(const int* g, int k, int mapf, int wtf, int* wto, int* sst, int* nc) {
  const int s = g[BFO_STRIDE], dw = g[BFO_DW], res = g[BFO_RES], wo = g[BFO_WO], ho = g[BFO_HO];
  *wto = 0;
  *sst = 0;
  if (k == 0) {
    const int H = g[BFO_H], W = g[BFO_W], cinp = g[BFO_CINP], kq = cinp / 4;
    const int band_nc = bfs_nc(4, g[BFO_NCT]);  // the band task is compiled for NC = 1
    const int wt_at = wtf - g[BFO_COUTP] * g[BFO_KS];
    if (dw && s == 2 && res == BF_RES_MAXPOOL && !g[BFO_PADT] && !g[BFO_PADL] && ho == 16 && wo == 16 &&
        H == 2 * ho && W == 2 * wo && band_nc == 1 && (H / 2 + 1) * W * kq <= BFS_BQ * BFS_NW * 64 &&
        (H / 2 + 1) * W * (cinp + 4) <= mapf + wt_at) {
      *wto = wt_at;
      *sst = cinp + 4;
      *nc = band_nc;
      return BFV_BAND;
    }
    return BFV_GLOBAL;
  }
  if (!dw) return BFV_HEAD;
  if (res == BF_RES_MAXPOOL) return BFV_MP;
  if (s == 1 && (wo == 16 || wo == 8) && g[BFO_W] == wo && g[BFO_PADL] == 1) return wo == 16 ? BFV_DPP16 : BFV_DPP8;
  return BFV_S1;
}

static int check_stage(const int* f, int i, int rest) {
  const int ni = f[BFO_NI], cs = f[BFO_CS], mapf = f[BFO_ROWS], wtf = f[BFO_COLS], lds = f[BFO_LDS];
  if (ni < 1 || ni > BFS_MAX || ni > rest) return hpe_fail(HPE_EINVAL, "blazeface stage %d: %d ops (max %d, %d follow)", i, ni, BFS_MAX, rest);
  if (cs < 8 || cs % 4 || mapf < 0 || mapf % 4 || wtf < 0 || wtf % 4 || lds > 160 * 1024 || lds < 4 * (mapf + wtf))
    return hpe_fail(HPE_EINVAL, "blazeface stage %d: LDS geometry", i);
  const int dwf = lds / 4 - mapf - wtf;
  int last_dst = -1;
  for (int k = 0; k < ni; ++k) {
    const int* g = f + (k + 1) * BFO_WORDS;
    const int kind = g[BFO_KIND], dw = g[BFO_DW], s = g[BFO_STRIDE];
    const int ho = g[BFO_HO], wo = g[BFO_WO], h = g[BFO_H], w = g[BFO_W], cinp = g[BFO_CINP], coutp = g[BFO_COUTP];
    if (kind != BF_BLOCK && kind != BF_DIRECT) return hpe_fail(HPE_EINVAL, "blazeface stage %d op %d: kind %d", i, k, kind);
    if (wo <= 0 || (wo & (wo - 1)) || (ho * wo) % 32 || ho * wo > 32 * BFS_NW || g[BFO_NCT] > 4 ||
        !bfs_nc((ho * wo) >> 5, g[BFO_NCT]))
      return hpe_fail(HPE_EINVAL, "blazeface stage %d op %d: map / channel-chunk geometry", i, k);
    if ((coutp + (dw ? 10 : 0)) * (cinp / 4) > BFS_PF * BFS_NW * 64 || coutp * g[BFO_KS] > wtf || (dw && 10 * cinp > dwf))
      return hpe_fail(HPE_EINVAL, "blazeface stage %d op %d: weights exceed the stage's share", i, k);
    if (dw ? (g[BFO_RES] != BF_RES_ID && g[BFO_RES] != BF_RES_MAXPOOL) || !g[BFO_RELU] : g[BFO_RELU])
      return hpe_fail(HPE_EINVAL, "blazeface stage %d op %d: residual / ReLU variant", i, k);
    if ((g[BFO_RES] == BF_RES_MAXPOOL && (s != 2 || h != 2 * ho || w != 2 * wo || g[BFO_PADT] || g[BFO_PADL])) ||
        (g[BFO_RES] == BF_RES_ID && (s != 1 || h != ho || w != wo)))
      return hpe_fail(HPE_EINVAL, "blazeface stage %d op %d: stride / residual geometry", i, k);
    if (k == 0) {
      if (!dw || g[BFO_SRC] == BF_BUF_IMG) return hpe_fail(HPE_EINVAL, "blazeface stage %d: must start with a block reading a map", i);
    } else {
      if (g[BFO_SRC] != last_dst || (h + 2) * w * (cinp + 4) > mapf || cinp + 4 > cs) return hpe_fail(HPE_EINVAL, "blazeface stage %d op %d: source is not the resident map", i, k);
      if (!dw && last_dst < BF_BUF_OUT0) return hpe_fail(HPE_EINVAL, "blazeface stage %d op %d: heads must read a tap", i, k);
    }
    if (dw) {
      if ((ho + 2) * wo * (coutp + 4) > mapf || coutp + 4 > cs) return hpe_fail(HPE_EINVAL, "blazeface stage %d op %d: output map exceeds LDS", i, k);
      if (g[BFO_SPLIT] || g[BFO_OSTRIDE] != coutp) return hpe_fail(HPE_EINVAL, "blazeface stage %d op %d: block output stride", i, k);
      last_dst = g[BFO_DST];
    } else if (g[BFO_RES] != BF_RES_NONE || g[BFO_DST] < BF_BUF_OUT0) {
      return hpe_fail(HPE_EINVAL, "blazeface stage %d op %d: heads geometry", i, k);
    }
  }
  return 0;
}

// the front record: its six records must be the BlazeFace backbone's stem and first five blocks as
// bf_front_kernel hard-codes them (BffL), chained through the workspace buffers
static int check_front(const int* f, int i, int rest) {
  if (f[BFO_NI] != 6 || rest < 6) return hpe_fail(HPE_EINVAL, "blazeface front %d: needs the stem + 5 block records", i);
  if (f[BFO_LDS] != 4 * BFF_FLOATS) return hpe_fail(HPE_EINVAL, "blazeface front %d: LDS %d != %d", i, f[BFO_LDS], 4 * BFF_FLOATS);
  const int* g = f + BFO_WORDS;
  if (g[BFO_KIND] != BF_STEM || g[BFO_H] != 128 || g[BFO_W] != 128 || g[BFO_HO] != 64 || g[BFO_WO] != 64 ||
      g[BFO_CIN] != 3 || g[BFO_COUT] != 24 || g[BFO_STRIDE] != 2 || g[BFO_PADT] != 1 || g[BFO_PADL] != 1 ||
      g[BFO_SRC] != BF_BUF_IMG)
    return hpe_fail(HPE_EINVAL, "blazeface front %d: stem geometry", i);
  struct { int s, cinp, coutp, h, ho, padt, res; } L[6] = {
      {0}, {1, 24, 24, 64, 64, 1, BF_RES_ID}, {1, 24, 32, 64, 64, 1, BF_RES_ID}, {2, 32, 32, 64, 32, 0, BF_RES_MAXPOOL},
      {1, 32, 40, 32, 32, 1, BF_RES_ID}, {1, 40, 48, 32, 32, 1, BF_RES_ID}};
  // bf_front_kernel keeps the stem's and blocks 1-4's maps in LDS rings (never in HBM): each of
  // them must go to a workspace buffer (not a caller output), and no record after the front may
  // read it (checked below over the rest of the plan)
  int last = g[BFO_DST];
  if (last != BF_BUF_A && last != BF_BUF_B) return hpe_fail(HPE_EINVAL, "blazeface front %d: stem output buffer", i);
  for (int k = 1; k <= 5; ++k) {
    const int* b = f + (k + 1) * BFO_WORDS;
    if ((b[BFO_KIND] != BF_ROWS && b[BFO_KIND] != BF_BLOCK) || !b[BFO_DW] || !b[BFO_RELU] || b[BFO_SPLIT] ||
        b[BFO_STRIDE] != L[k].s || b[BFO_CINP] != L[k].cinp || b[BFO_COUTP] != L[k].coutp || b[BFO_H] != L[k].h ||
        b[BFO_W] != L[k].h || b[BFO_HO] != L[k].ho || b[BFO_WO] != L[k].ho || b[BFO_PADT] != L[k].padt ||
        b[BFO_PADL] != L[k].padt || b[BFO_RES] != L[k].res || b[BFO_SRC] != last || b[BFO_OSTRIDE] != L[k].coutp)
      return hpe_fail(HPE_EINVAL, "blazeface front %d: block %d geometry", i, k);
    last = b[BFO_DST];
    if (last != BF_BUF_A && last != BF_BUF_B) return hpe_fail(HPE_EINVAL, "blazeface front %d: block %d output buffer", i, k);
  }
  // after the front only block 5's map is in a ping-pong buffer: the other buffer holds no map
  // until a later record writes it (a stage reads HBM in its first op only, its blocks' maps stay
  // in LDS: they write nothing)
  const int other = last == BF_BUF_A ? BF_BUF_B : BF_BUF_A;
  bool other_ok = false;
  for (int k = 7; k <= rest; ++k) {
    const int* r = f + k * BFO_WORDS;
    if (r[BFO_KIND] == BF_STAGE) {
      if (k + 1 <= rest && (r + BFO_WORDS)[BFO_SRC] == other && !other_ok)
        return hpe_fail(HPE_EINVAL, "blazeface front %d: record %d reads a map the front keeps in LDS", i, i + k + 1);
      k += r[BFO_NI];
      continue;
    }
    if (r[BFO_SRC] == other && !other_ok)
      return hpe_fail(HPE_EINVAL, "blazeface front %d: record %d reads a map the front keeps in LDS", i, i + k);
    if (r[BFO_DST] == other || (r[BFO_SPLIT] && r[BFO_DST2] == other)) other_ok = true;
  }
  return 0;
}

static int check_op(const int* f, int i, int rest) {
  const int kind = f[BFO_KIND];
  if (kind == BF_STAGE) return check_stage(f, i, rest);
  if (kind == BF_FRONT) return check_front(f, i, rest);
  if (kind != BF_STEM && kind != BF_BLOCK && kind != BF_ROWS && kind != BF_DIRECT) return hpe_fail(HPE_EINVAL, "blazeface op %d: bad kind %d", i, kind);
  if (kind == BF_DIRECT) {
    const int s = f[BFO_STRIDE], dw = f[BFO_DW], wo = f[BFO_WO], ho = f[BFO_HO];
    if (!pick_direct(s, dw, f[BFO_NC]) || f[BFO_NC] != f[BFO_NCT]) return hpe_fail(HPE_EINVAL, "blazeface op %d: no direct kernel S=%d DW=%d NC=%d", i, s, dw, f[BFO_NC]);
    if (wo <= 0 || (wo & (wo - 1)) || (ho * wo) % 32) return hpe_fail(HPE_EINVAL, "blazeface op %d: direct kernel needs Wo a power of two, Ho*Wo % 32 == 0", i);
    if (f[BFO_WAVES] < 1 || f[BFO_WAVES] > 4) return hpe_fail(HPE_EINVAL, "blazeface op %d: waves", i);
    if (f[BFO_CINP] % 8 || f[BFO_CINP] < f[BFO_CIN] || f[BFO_COUTP] % 8 || f[BFO_COUTP] < f[BFO_COUT] ||
        f[BFO_KS] < f[BFO_CINP] || f[BFO_KS] % 4 || f[BFO_NCT] < 1 || f[BFO_NCT] * 32 < f[BFO_COUTP])
      return hpe_fail(HPE_EINVAL, "blazeface op %d: channel geometry", i);
    if (dw ? (s == 1 ? (f[BFO_H] != ho || f[BFO_W] != wo || f[BFO_PADT] != 1 || f[BFO_PADL] != 1)
                     : (f[BFO_H] != 2 * ho || f[BFO_W] != 2 * wo || f[BFO_PADT] || f[BFO_PADL]))
           : (f[BFO_H] != ho || f[BFO_W] != wo || s != 1))
      return hpe_fail(HPE_EINVAL, "blazeface op %d: direct kernel map geometry", i);
    if ((f[BFO_RES] == BF_RES_MAXPOOL && s != 2) || (f[BFO_RES] == BF_RES_ID && s != 1))
      return hpe_fail(HPE_EINVAL, "blazeface op %d: residual / stride", i);
    const long need = 4L * (f[BFO_NCT] * 32 * f[BFO_KS] + (dw ? 10 * f[BFO_CINP] : 0));
    if (f[BFO_LDS] < need || f[BFO_LDS] > 160 * 1024) return hpe_fail(HPE_EINVAL, "blazeface op %d: LDS", i);
    if (f[BFO_SRC] < 0 || f[BFO_SRC] >= BF_NBUF || f[BFO_DST] < 0 || f[BFO_DST] >= BF_NBUF) return hpe_fail(HPE_EINVAL, "blazeface op %d: bad buffer", i);
    if (!f[BFO_SPLIT] && (f[BFO_OSTRIDE] < f[BFO_COUT] || f[BFO_OSTRIDE] > f[BFO_COUTP]))
      return hpe_fail(HPE_EINVAL, "blazeface op %d: output stride", i);
    if (f[BFO_SPLIT] && (f[BFO_DST2] < 0 || f[BFO_DST2] >= BF_NBUF || f[BFO_SPLIT] >= f[BFO_COUT]))
      return hpe_fail(HPE_EINVAL, "blazeface op %d: bad split", i);
    return 0;
  }
  if (kind == BF_ROWS) {
    const int S = f[BFO_STRIDE], R = f[BFO_TH], nseg = f[BFO_NI], kq = f[BFO_CINP] / 4;
    if (!pick_rows_op(f) || !f[BFO_DW] || f[BFO_SPLIT] || !f[BFO_RELU]) return hpe_fail(HPE_EINVAL, "blazeface op %d: rows kernel variant", i);
    if (f[BFO_WAVES] < 1 || f[BFO_WAVES] > 4) return hpe_fail(HPE_EINVAL, "blazeface op %d: waves", i);
    if (R <= 0 || nseg <= 0 || f[BFO_HO] % nseg || (f[BFO_HO] / nseg) % R) return hpe_fail(HPE_EINVAL, "blazeface op %d: row steps", i);
    const int wo = f[BFO_WO];
    if (wo < 16 || (wo & (wo - 1)) || (R * wo) % 32) return hpe_fail(HPE_EINVAL, "blazeface op %d: rows kernel needs Wo >= 16, a power of two", i);
    if (f[BFO_ROWS] != (R - 1) * S + 3 || f[BFO_COLS] != (wo - 1) * S + 3) return hpe_fail(HPE_EINVAL, "blazeface op %d: ring geometry", i);
    if (S == 1 ? (f[BFO_PADT] != 1 || f[BFO_PADL] != 1 || f[BFO_RES] != BF_RES_ID || f[BFO_H] != f[BFO_HO] || f[BFO_W] != wo)
               : (f[BFO_PADT] || f[BFO_PADL] || f[BFO_RES] != BF_RES_MAXPOOL || f[BFO_H] != 2 * f[BFO_HO] || f[BFO_W] != 2 * wo))
      return hpe_fail(HPE_EINVAL, "blazeface op %d: rows kernel stride/padding/residual", i);
    if (R * S * f[BFO_W] * kq > RPF * 64 * f[BFO_WAVES]) return hpe_fail(HPE_EINVAL, "blazeface op %d: prefetch share exceeds %d float4/thread", i, RPF);
    if (f[BFO_CINP] % 8 || f[BFO_CS] < f[BFO_CINP] || f[BFO_CS] % 4 || f[BFO_KS] < f[BFO_CINP] || f[BFO_KS] % 4 ||
        f[BFO_NCT] < 1 || f[BFO_NCT] * 32 < f[BFO_COUTP] || f[BFO_NCT] % f[BFO_NC] || f[BFO_OSTRIDE] < f[BFO_COUT] ||
        f[BFO_OSTRIDE] > f[BFO_COUTP] || f[BFO_COUTP] % 8)
      return hpe_fail(HPE_EINVAL, "blazeface op %d: channel geometry", i);
    const long need = 4L * (f[BFO_NCT] * 32 * f[BFO_KS] + 10 * f[BFO_CINP] + (long)f[BFO_ROWS] * f[BFO_COLS] * f[BFO_CS]);
    if (f[BFO_LDS] < need || f[BFO_LDS] > 160 * 1024) return hpe_fail(HPE_EINVAL, "blazeface op %d: LDS", i);
    if (f[BFO_SRC] < 0 || f[BFO_SRC] >= BF_NBUF || f[BFO_DST] < 0 || f[BFO_DST] >= BF_NBUF) return hpe_fail(HPE_EINVAL, "blazeface op %d: bad buffer", i);
    return 0;
  }
  if (f[BFO_TH] <= 0 || f[BFO_NI] <= 0 || f[BFO_HO] % f[BFO_TH]) return hpe_fail(HPE_EINVAL, "blazeface op %d: bad tile", i);
  if ((f[BFO_NI] * f[BFO_TH] * f[BFO_WO]) % 32) return hpe_fail(HPE_EINVAL, "blazeface op %d: tile not a multiple of 32 positions", i);
  if (f[BFO_NI] > 1 && f[BFO_TH] != f[BFO_HO]) return hpe_fail(HPE_EINVAL, "blazeface op %d: multi-image tiles must be whole images", i);
  if (f[BFO_LDS] <= 0 || f[BFO_LDS] > 160 * 1024) return hpe_fail(HPE_EINVAL, "blazeface op %d: LDS %d bytes", i, f[BFO_LDS]);
  if (f[BFO_SRC] < 0 || f[BFO_SRC] >= BF_NBUF || f[BFO_DST] < 0 || f[BFO_DST] >= BF_NBUF)
    return hpe_fail(HPE_EINVAL, "blazeface op %d: bad buffer", i);
  const int wo = f[BFO_WO], ppi = f[BFO_TH] * f[BFO_WO];
  if (wo <= 0 || (wo & (wo - 1)) || (ppi & (ppi - 1))) return hpe_fail(HPE_EINVAL, "blazeface op %d: Wo and TH*Wo must be powers of two", i);
  if (f[BFO_WAVES] < 1 || f[BFO_WAVES] > (kind == BF_STEM ? 4 : 8)) return hpe_fail(HPE_EINVAL, "blazeface op %d: waves", i);
  if (kind == BF_STEM) {
    if (f[BFO_CIN] != 3 || f[BFO_COUT] > 32 || f[BFO_STRIDE] != 2) return hpe_fail(HPE_EINVAL, "blazeface stem: unsupported geometry");
    const int rows = 2 * (f[BFO_TH] - 1) + 6, cols = 2 * (f[BFO_WO] - 1) + 5;
    if (f[BFO_ROWS] != rows || f[BFO_COLS] != cols || f[BFO_LDS] < rows * cols * 12)
      return hpe_fail(HPE_EINVAL, "blazeface stem: tile words inconsistent");
    return 0;
  }
  const int s = f[BFO_STRIDE], dw = f[BFO_DW];
  if (f[BFO_NCT] < 1 || f[BFO_NCT] * 32 < f[BFO_COUTP] || f[BFO_NCT] % f[BFO_NC] || f[BFO_CINP] / 4 > 64 * f[BFO_WAVES])
    return hpe_fail(HPE_EINVAL, "blazeface op %d: channel chunks", i);
  if (!pick_block(s, dw, f[BFO_NC])) return hpe_fail(HPE_EINVAL, "blazeface op %d: no kernel for S=%d DW=%d NC=%d", i, s, dw, f[BFO_NC]);
  if (f[BFO_CINP] % 8 || f[BFO_CINP] < f[BFO_CIN] || f[BFO_COUTP] % 8 || f[BFO_COUTP] < f[BFO_COUT] ||
      f[BFO_CS] < f[BFO_CINP] || f[BFO_CS] % 4 || f[BFO_KS] < f[BFO_CINP] || f[BFO_KS] % 4)
    return hpe_fail(HPE_EINVAL, "blazeface op %d: channel geometry", i);
  const int rows = dw ? (f[BFO_TH] - 1) * s + 3 : f[BFO_TH];
  const int cols = dw ? (f[BFO_WO] - 1) * s + 3 : f[BFO_WO];
  if (f[BFO_ROWS] != rows || f[BFO_COLS] != cols) return hpe_fail(HPE_EINVAL, "blazeface op %d: tile rows/cols", i);
  if (f[BFO_RES] == BF_RES_MAXPOOL && (s != 2 || f[BFO_H] % 2 || f[BFO_W] % 2 || f[BFO_PADT] || f[BFO_PADL]))
    return hpe_fail(HPE_EINVAL, "blazeface op %d: maxpool residual needs s2 on even maps", i);
  if (f[BFO_RES] == BF_RES_ID && s != 1) return hpe_fail(HPE_EINVAL, "blazeface op %d: identity residual needs s1", i);
  const long need = 4L * (f[BFO_NCT] * 32 * f[BFO_KS] + (dw ? 10 * f[BFO_CINP] : 0) +
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
    const int rc = check_op(words + off + i * BFO_WORDS, i, nops - 1 - i);
    if (rc) return rc;
  }
  hpe_blazeface* h = (hpe_blazeface*)calloc(1, sizeof(hpe_blazeface));
  h->words = (int*)malloc(sizeof(int) * n_words);
  memcpy(h->words, words, sizeof(int) * n_words);
  h->n_words = (int)n_words;
  h->nops = nops;
  h->act_floats = words[BFH_ACT_FLOATS];
  int dev = 0, ncu = 256;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  h->n_cu = ncu > 0 ? ncu : 256;
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
    if (f[BFO_KIND] == BF_FRONT) {  // the stem + five blocks as one launch, one workgroup per frame
      BfFrontArgs fa;
      memset(&fa, 0, sizeof fa);
      memcpy(fa.stem, f + BFO_WORDS, sizeof fa.stem);
      for (int k = 1; k <= 5; ++k) {
        const int* b = f + (k + 1) * BFO_WORDS;
        fa.dww[k] = b[BFO_DWW];
        fa.pww[k] = b[BFO_PWW];
        fa.pwb[k] = b[BFO_PWB];
      }
      fa.params = params;
      fa.src = bufs[BF_BUF_IMG];
      fa.dst = bufs[(f + 6 * BFO_WORDS)[BFO_DST]];
      fa.nimg = n_images;
      const int64_t grid = n_images < h->n_cu ? n_images : h->n_cu;
      hipFuncSetAttribute((const void*)bf_front_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 4 * BFF_FLOATS);
      hipLaunchKernelGGL(bf_front_kernel, dim3((unsigned)grid), dim3(BFF_NW * 64), 4 * BFF_FLOATS, s, fa);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return hpe_fail(HPE_ERUNTIME, "blazeface front %d launch: %s", i, hipGetErrorString(e));
      i += f[BFO_NI];
      continue;
    }
    if (f[BFO_KIND] == BF_STAGE) {  // the next BFO_NI records as one launch, one workgroup per image
      if (n_images > 0x7fffffff) return hpe_fail(HPE_EINVAL, "blazeface_forward: batch too large");
      BfStageArgs sa;
      memset(&sa, 0, sizeof sa);
      const int ni = f[BFO_NI];
      sa.nops = ni;
      sa.map_floats = f[BFO_ROWS];
      sa.wt_floats = f[BFO_COLS];
      sa.params = params;
      for (int b = 0; b < BF_NBUF; ++b) sa.bufs[b] = bufs[b];
      for (int k = 0; k < ni; ++k) {
        const int* g = f + (k + 1) * BFO_WORDS;
        BfSub& o = sa.op[k];
        o.s = g[BFO_STRIDE]; o.h = g[BFO_H]; o.w = g[BFO_W]; o.ho = g[BFO_HO]; o.wo = g[BFO_WO];
        o.cin = g[BFO_CIN]; o.cinp = g[BFO_CINP]; o.cout = g[BFO_COUT]; o.coutp = g[BFO_COUTP];
        o.ks = g[BFO_KS]; o.nct = g[BFO_NCT]; o.nc = bfs_nc_run((o.ho * o.wo) >> 5, o.nct);
        o.res = g[BFO_RES]; o.relu = g[BFO_RELU]; o.dw = g[BFO_DW]; o.padt = g[BFO_PADT]; o.padl = g[BFO_PADL];
        o.dww = g[BFO_DWW]; o.pww = g[BFO_PWW]; o.pwb = g[BFO_PWB];
        o.var = bfs_variant(g, k, sa.map_floats, sa.wt_floats, &o.wto, &o.sst, &o.nc);
        o.ss = o.cinp + 4;
        o.cso = o.coutp + 4;
        // the first op's map replaces the staged rows / the source in global memory; a block whose
        // output map differs in shape or stride from its source gets fresh halo rows
        o.zhalo = g[BFO_DW] && (k == 0 || o.ho != o.h || o.wo != o.w || o.cso != o.ss);
        if (k == 0) sa.src = bufs[g[BFO_SRC]];
        o.lds_out = g[BFO_DW] ? 1 : 0;
        o.gdst = g[BFO_DW] ? (g[BFO_DST] >= BF_BUF_OUT0 ? g[BFO_DST] : -1) : g[BFO_DST];
        o.split = g[BFO_SPLIT];
        o.gdst2 = o.split ? g[BFO_DST2] : -1;
        o.ostride = g[BFO_OSTRIDE];
      }
      hipFuncSetAttribute((const void*)bf_stage_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, f[BFO_LDS]);
      hipLaunchKernelGGL(bf_stage_kernel, dim3((unsigned)n_images), dim3(BFS_NW * 64), f[BFO_LDS], s, sa);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return hpe_fail(HPE_ERUNTIME, "blazeface stage %d launch: %s", i, hipGetErrorString(e));
      i += ni;
      continue;
    }
    BfArgs a;
    memcpy(a.f, f, sizeof a.f);
    a.params = params;
    a.src = bufs[f[BFO_SRC]];
    a.dst = bufs[f[BFO_DST]];
    a.dst2 = f[BFO_SPLIT] ? bufs[f[BFO_DST2]] : nullptr;
    a.nimg = n_images;
    const int64_t tpi = f[BFO_TH] > 0 ? f[BFO_HO] / f[BFO_TH] : 1;
    const int threads = 64 * f[BFO_WAVES];
    bf_fn k = f[BFO_KIND] == BF_STEM ? bf_stem_kernel
              : f[BFO_KIND] == BF_ROWS ? pick_rows_op(f)
              : f[BFO_KIND] == BF_DIRECT ? pick_direct(f[BFO_STRIDE], f[BFO_DW], f[BFO_NC])
                                       : pick_block(f[BFO_STRIDE], f[BFO_DW], f[BFO_NC]);
    hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, f[BFO_LDS]);
    int64_t nwg;
    if (f[BFO_KIND] == BF_DIRECT) {  // persistent: as many workgroups as fit, capped by the tasks
      const int64_t tasks = n_images * ((f[BFO_HO] * f[BFO_WO]) >> 5);
      int per_cu = (160 * 1024) / f[BFO_LDS];
      if (per_cu > 12 / f[BFO_WAVES]) per_cu = 12 / f[BFO_WAVES];
#ifndef BF_NO_OCC
      // resident workgroups as the runtime counts them (VGPRs + AGPRs, LDS): a grid sized past
      // them runs its tasks in a second, partial round
      int res = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&res, (const void*)k, threads, f[BFO_LDS]) == hipSuccess &&
          res > 0 && per_cu > res)
        per_cu = res;
#endif
      if (per_cu < 1) per_cu = 1;
      nwg = (tasks + f[BFO_WAVES] - 1) / f[BFO_WAVES];
      if (nwg > (int64_t)h->n_cu * per_cu) nwg = (int64_t)h->n_cu * per_cu;
    } else {
      nwg = f[BFO_KIND] == BF_ROWS ? n_images * f[BFO_NI]
            : f[BFO_NI] > 1 ? (n_images + f[BFO_NI] - 1) / f[BFO_NI] : n_images * tpi;
    }
    if (nwg > 0x7fffffff) return hpe_fail(HPE_EINVAL, "blazeface_forward: batch too large");
    a.nwg = (int)nwg;
    hipLaunchKernelGGL(k, dim3((unsigned)nwg), dim3(threads), f[BFO_LDS], s, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hpe_fail(HPE_ERUNTIME, "blazeface op %d launch: %s", i, hipGetErrorString(e));
  }
  return HPE_OK;
}
