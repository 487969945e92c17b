// hpe_detect.hip — batched detector post-processing of the unified BlazeFace graph
// (blazeFaceDetectorH5.py:271-357), one workgroup per frame:
//   filterDetections   logit > log(t / (1 - t)) in fp32, score = 1 / (1 + exp(-logit))      :319-327
//   extractDetections  anchor decode in fp64 (anchors: blazeFaceUtils.gen_anchors with the
//                      detector's options: 16x16 x 2 + 8x8 x 6 centres, fixed size)        :284-317
//   NMS                tf.image.non_max_suppression (V3): greedy by score (ties: lower index),
//                      IoU in fp32 on the fp32-cast boxes, suppress iff IoU > threshold    :332
//   pose gather        detection index -> pose cell of the 16x16 / 8x8 regressor map       :342-353
// Candidates are compacted and bitonic-sorted in LDS (64-bit keys: ordered score, ~index); the
// greedy pass suppresses in parallel across the workgroup, one barrier pair per kept box.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hpe.h"
#include "hpe_common.h"

#define DET_N0 512      // 16 x 16 cells x 2 anchors (stride 8)
#define DET_N1 384      // 8 x 8 cells x 6 anchors (strides 16, 16, 16 merged)
#define DET_N 896
#define DET_SORT 1024
#define DET_KP 6
#define DET_LOC 16
#define DET_T 256

struct DetArgs {
  const float *cls0, *cls1, *loc0, *loc1, *pose0, *pose1;
  float thr, iou;
  int max_faces;
  int32_t* count;
  int32_t* det_index;
  float* scores;
  double* boxes;
  double* keypoints;
  float* poses;
};

__device__ __forceinline__ uint32_t f2ord(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ void anchor_center(int d, double* ax, double* ay) {
  if (d < DET_N0) {
    const int cell = d >> 1;
    *ax = ((cell & 15) + 0.5) / 16.0;
    *ay = ((cell >> 4) + 0.5) / 16.0;
  } else {
    const int cell = (d - DET_N0) / 6;
    *ax = ((cell & 7) + 0.5) / 8.0;
    *ay = ((cell >> 3) + 0.5) / 8.0;
  }
}

__global__ void __launch_bounds__(DET_T) detect_kernel(DetArgs a) {
  __shared__ uint64_t key[DET_SORT];
  __shared__ float fb[DET_N][4];        // fp32 boxes (NMS input), by detection index
  __shared__ int sup[DET_SORT];
  __shared__ int ncand, nsel, cur_keep;
  const int64_t img = blockIdx.x;
  const int t = threadIdx.x;
  if (t == 0) {
    ncand = 0;
    nsel = 0;
  }
  for (int i = t; i < DET_SORT; i += DET_T) {
    key[i] = 0;
    sup[i] = 0;
  }
  __syncthreads();
  // ---- threshold + compaction ----
  for (int d = t; d < DET_N; d += DET_T) {
    const float logit = d < DET_N0 ? a.cls0[img * DET_N0 + d] : a.cls1[img * DET_N1 + d - DET_N0];
    if (logit > a.thr) {
      const float sc = 1.0f / (1.0f + expf(-logit));
      const int slot = atomicAdd(&ncand, 1);
      key[slot] = ((uint64_t)f2ord(sc) << 32) | (uint32_t)(0xFFFFFFFFu - (uint32_t)d);
      const float* lp = d < DET_N0 ? a.loc0 + (img * DET_N0 + d) * DET_LOC : a.loc1 + (img * DET_N1 + d - DET_N0) * DET_LOC;
      double ax, ay;
      anchor_center(d, &ax, &ay);
      const double cx = ((double)lp[0] + ax * 128.0) / 128.0;
      const double cy = ((double)lp[1] + ay * 128.0) / 128.0;
      const double w = (double)lp[2] / 128.0, h = (double)lp[3] / 128.0;
      fb[d][0] = (float)(cx - w * 0.5);
      fb[d][1] = (float)(cy - h * 0.5);
      fb[d][2] = (float)(cx + w * 0.5);
      fb[d][3] = (float)(cy + h * 0.5);
    }
  }
  __syncthreads();
  const int n = ncand;
  // ---- bitonic sort, descending (score desc, then index asc) ----
  for (int k = 2; k <= DET_SORT; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = t; i < DET_SORT; i += DET_T) {
        const int p = i ^ j;
        if (p > i) {
          const uint64_t x = key[i], y = key[p];
          const bool desc = (i & k) == 0;
          if (desc ? (x < y) : (x > y)) {
            key[i] = y;
            key[p] = x;
          }
        }
      }
      __syncthreads();
    }
  }
  // ---- greedy NMS ----
  for (int i = 0; i < n; ++i) {
    if (nsel >= a.max_faces) break;   // uniform: read after the barrier below
    if (sup[i]) continue;             // uniform
    const int di = (int)(0xFFFFFFFFu - (uint32_t)key[i]);
    if (t == 0) {
      cur_keep = nsel;
      const int64_t o = img * a.max_faces + nsel;
      a.det_index[o] = di;
      a.scores[o] = __uint_as_float((uint32_t)(key[i] >> 32) & 0x80000000u ? (uint32_t)(key[i] >> 32) & 0x7FFFFFFFu
                                                                             : ~(uint32_t)(key[i] >> 32));
    }
    const float ymin_i = fminf(fb[di][0], fb[di][2]), xmin_i = fminf(fb[di][1], fb[di][3]);
    const float ymax_i = fmaxf(fb[di][0], fb[di][2]), xmax_i = fmaxf(fb[di][1], fb[di][3]);
    const float area_i = (ymax_i - ymin_i) * (xmax_i - xmin_i);
    for (int j = i + 1 + t; j < n; j += DET_T) {
      if (sup[j]) continue;
      const int dj = (int)(0xFFFFFFFFu - (uint32_t)key[j]);
      const float ymin_j = fminf(fb[dj][0], fb[dj][2]), xmin_j = fminf(fb[dj][1], fb[dj][3]);
      const float ymax_j = fmaxf(fb[dj][0], fb[dj][2]), xmax_j = fmaxf(fb[dj][1], fb[dj][3]);
      const float area_j = (ymax_j - ymin_j) * (xmax_j - xmin_j);
      float iou = 0.f;
      if (area_i > 0.f && area_j > 0.f) {
        const float iy0 = fmaxf(ymin_i, ymin_j), ix0 = fmaxf(xmin_i, xmin_j);
        const float iy1 = fminf(ymax_i, ymax_j), ix1 = fminf(xmax_i, xmax_j);
        const float inter = fmaxf(iy1 - iy0, 0.f) * fmaxf(ix1 - ix0, 0.f);
        iou = inter / (area_i + area_j - inter);
      }
      if (iou > a.iou) sup[j] = 1;
    }
    __syncthreads();
    if (t == 0) nsel = nsel + 1;
    __syncthreads();
  }
  __syncthreads();
  const int ns = nsel;
  if (t == 0) a.count[img] = ns;
  // ---- fp64 boxes / keypoints and pose gather for the kept detections ----
  for (int s = t; s < ns; s += DET_T) {
    const int64_t o = img * a.max_faces + s;
    const int d = a.det_index[o];
    const float* lp = d < DET_N0 ? a.loc0 + (img * DET_N0 + d) * DET_LOC : a.loc1 + (img * DET_N1 + d - DET_N0) * DET_LOC;
    double ax, ay;
    anchor_center(d, &ax, &ay);
    const double cx = ((double)lp[0] + ax * 128.0) / 128.0;
    const double cy = ((double)lp[1] + ay * 128.0) / 128.0;
    const double w = (double)lp[2] / 128.0, h = (double)lp[3] / 128.0;
    double* bo = a.boxes + o * 4;
    bo[0] = cx - w * 0.5;
    bo[1] = cy - h * 0.5;
    bo[2] = cx + w * 0.5;
    bo[3] = cy + h * 0.5;
    double* ko = a.keypoints + o * DET_KP * 2;
    for (int j = 0; j < DET_KP; ++j) {
      ko[2 * j] = ((double)lp[4 + 2 * j] + ax * 128.0) / 128.0;
      ko[2 * j + 1] = ((double)lp[5 + 2 * j] + ay * 128.0) / 128.0;
    }
    const float* pp;
    if (d < DET_N0) {
      const int cell = d >> 1;
      pp = a.pose0 + (img * 256 + cell) * 3;
    } else {
      const int cell = (d - DET_N0) / 6;
      pp = a.pose1 + (img * 64 + cell) * 3;
    }
    float* po = a.poses + o * 3;
    po[0] = pp[0];
    po[1] = pp[1];
    po[2] = pp[2];
  }
}

extern "C" int hpe_detect(const float* cls0, const float* cls1, const float* loc0, const float* loc1,
                          const float* pose0, const float* pose1, int64_t n_images, float score_logit_threshold,
                          float iou_threshold, int32_t max_faces, int32_t* count, int32_t* det_index,
                          float* scores, double* boxes, double* keypoints, float* poses, void* stream) {
  if (!cls0 || !cls1 || !loc0 || !loc1 || !pose0 || !pose1 || !count || !det_index || !scores || !boxes ||
      !keypoints || !poses)
    return hpe_fail(HPE_EINVAL, "hpe_detect: null argument");
  if (max_faces <= 0) return hpe_fail(HPE_EINVAL, "hpe_detect: max_faces must be positive");
  if (n_images <= 0) return HPE_OK;
  if (n_images > 0x7fffffff) return hpe_fail(HPE_EINVAL, "hpe_detect: batch too large");
  DetArgs a = {cls0, cls1, loc0, loc1, pose0, pose1, score_logit_threshold, iou_threshold, (int)max_faces,
               count, det_index, scores, boxes, keypoints, poses};
  hipLaunchKernelGGL(detect_kernel, dim3((unsigned)n_images), dim3(DET_T), 0, (hipStream_t)stream, a);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hpe_fail(HPE_ERUNTIME, "hpe_detect launch: %s", hipGetErrorString(e));
  return HPE_OK;
}

// ---- feature-dataset extraction ------------------------------------------------
// For each of the first k kept detections of a frame, the regressor input its pose came from
// (blazeFaceDetectorH5.py:342-353): detection d < 512 -> re_lu_10 cell d / 2 of the 16 x 16 tap,
// otherwise re_lu_15 cell (d - 512) / 6 of the 8 x 8 tap.  One workgroup per (frame, slot), one
// float4 per lane (C0, C1 multiples of 4); the unused tap's row and empty slots are zero-filled and
// src = 0 (front) / 1 (back) / -1 (no detection).
__global__ void __launch_bounds__(64) gather_features_kernel(const int32_t* count, const int32_t* det_index,
                                                               int max_faces, int k, const float* tap0, int c0,
                                                               const float* tap1, int c1, float* feat0,
                                                               float* feat1, int32_t* src) {
  const int64_t img = blockIdx.x / k;
  const int j = blockIdx.x - (int)(img * k);
  const int t = threadIdx.x;
  const int64_t o = img * k + j;
  const int ns = count[img];
  int d = -1;
  if (j < ns) d = det_index[img * max_faces + j];
  const float4* s0 = nullptr;
  const float4* s1 = nullptr;
  if (d >= 0 && d < DET_N0) s0 = (const float4*)(tap0 + (img * 256 + (d >> 1)) * c0);
  if (d >= DET_N0) s1 = (const float4*)(tap1 + (img * 64 + (d - DET_N0) / 6) * c1);
  float4* f0 = (float4*)(feat0 + o * c0);
  float4* f1 = (float4*)(feat1 + o * c1);
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int i = t; i < c0 / 4; i += 64) f0[i] = s0 ? s0[i] : z;
  for (int i = t; i < c1 / 4; i += 64) f1[i] = s1 ? s1[i] : z;
  if (t == 0) src[o] = d < 0 ? -1 : (d < DET_N0 ? 0 : 1);
}

extern "C" int hpe_gather_features(const int32_t* count, const int32_t* det_index, int64_t n_images,
                                   int32_t max_faces, int32_t k, const float* tap0, int32_t c0, const float* tap1,
                                   int32_t c1, float* feat0, float* feat1, int32_t* src, void* stream) {
  if (!count || !det_index || !tap0 || !tap1 || !feat0 || !feat1 || !src)
    return hpe_fail(HPE_EINVAL, "hpe_gather_features: null argument");
  if (max_faces <= 0 || k <= 0 || k > max_faces)
    return hpe_fail(HPE_EINVAL, "hpe_gather_features: need 0 < k <= max_faces (k %d, max_faces %d)", k, max_faces);
  if (c0 <= 0 || c1 <= 0 || (c0 & 3) || (c1 & 3))
    return hpe_fail(HPE_EINVAL, "hpe_gather_features: channel counts %d / %d must be positive multiples of 4", c0, c1);
  if (n_images <= 0) return HPE_OK;
  if (n_images * k > 0x7fffffff) return hpe_fail(HPE_EINVAL, "hpe_gather_features: batch too large");
  hipLaunchKernelGGL(gather_features_kernel, dim3((unsigned)(n_images * k)), dim3(64), 0, (hipStream_t)stream,
                     count, det_index, (int)max_faces, (int)k, tap0, (int)c0, tap1, (int)c1, feat0, feat1, src);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hpe_fail(HPE_ERUNTIME, "hpe_gather_features launch: %s", hipGetErrorString(e));
  return HPE_OK;
}
