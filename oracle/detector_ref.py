"""CPU restatement of the BlazeFace detector post-processing — TEST INFRASTRUCTURE (oracle).

Follows BlazePoser/blazeFaceDetectorH5.py (reference file:line):
  __init__            sigmoidScoreThreshold = log(t / (1 - t))                         :82-85
  generateAnchors     SSD anchors, options of :232-239 via blazeFaceUtils.gen_anchors  :59-127
  inference           outputs -> loc/cls concatenated front (512) then back (384)      :271-282
  extractDetections   fp64 anchor decode of boxes and 6 keypoints                      :284-317
  filterDetections    fp32 threshold + fp32 sigmoid                                    :319-327
  filterWithNonMaxSupression  tf.image.non_max_suppression (V3 semantics restated: greedy by
                      score, ties to the lower index, fp32 IoU on fp32-cast boxes, suppress iff
                      IoU > threshold, at most MAX_FACE_NUM) + pose-cell gather          :329-357
tf.image.non_max_suppression is TensorFlow 2.13 (requirements.txt:2), absent here: its published
kernel semantics (non_max_suppression_op.cc, IOU + greedy selection) are restated below.  Anchors
are pinned against the reference's own generator (tests/golden/anchors_blazeface_128.npy, made by
tests/golden/make_anchor_fixture.py); NMS/decode parity beyond that is restatement-pinned.
"""
import math

import numpy as np

KEY_POINT_SIZE = 6     # blazeFaceDetectorH5.py:8
MAX_FACE_NUM = 100     # blazeFaceDetectorH5.py:9
INPUT = 128


def anchors():
    """(896, 4) [x_center, y_center, h, w]: gen_anchors with strides [8, 16, 16, 16], one aspect
    ratio + the interpolated one, fixed anchor size (blazeFaceUtils.py:59-127 restated)."""
    out = []
    strides = [8, 16, 16, 16]
    layer = 0
    while layer < len(strides):
        n_same = 0
        last = layer
        while last < len(strides) and strides[last] == strides[layer]:
            n_same += 2          # aspect 1.0 + interpolated scale
            last += 1
        fm = math.ceil(INPUT / strides[layer])
        for y in range(fm):
            for x in range(fm):
                for _ in range(n_same):
                    out.append(((x + 0.5) / fm, (y + 0.5) / fm, 1.0, 1.0))
        layer = last
    return np.asarray(out, dtype=np.float64)


def score_logit_threshold(score_threshold=0.4):
    return float(np.log(score_threshold / (1 - score_threshold)))


def _iou(bi, bj):
    """tf NMS IOU on fp32 boxes (corner order agnostic)."""
    f = np.float32
    ymin_i, xmin_i = min(bi[0], bi[2]), min(bi[1], bi[3])
    ymax_i, xmax_i = max(bi[0], bi[2]), max(bi[1], bi[3])
    ymin_j, xmin_j = min(bj[0], bj[2]), min(bj[1], bj[3])
    ymax_j, xmax_j = max(bj[0], bj[2]), max(bj[1], bj[3])
    area_i = f(f(ymax_i - ymin_i) * f(xmax_i - xmin_i))
    area_j = f(f(ymax_j - ymin_j) * f(xmax_j - xmin_j))
    if area_i <= 0 or area_j <= 0:
        return f(0)
    iy0, ix0 = max(ymin_i, ymin_j), max(xmin_i, xmin_j)
    iy1, ix1 = min(ymax_i, ymax_j), min(xmax_i, xmax_j)
    inter = f(max(f(iy1 - iy0), f(0)) * max(f(ix1 - ix0), f(0)))
    return f(inter / f(f(area_i + area_j) - inter))


def non_max_suppression(boxes, scores, max_output_size, iou_threshold):
    b = np.asarray(boxes, dtype=np.float32)
    s = np.asarray(scores, dtype=np.float32)
    order = sorted(range(len(s)), key=lambda i: (-float(s[i]), i))
    thr = np.float32(iou_threshold)
    sel = []
    for i in order:
        if len(sel) >= max_output_size:
            break
        if all(_iou(b[i], b[j]) <= thr for j in sel):
            sel.append(i)
    return np.asarray(sel, dtype=np.int64)


def detect_frame(cls0, cls1, loc0, loc1, pose_front, pose_back, score_threshold=0.4, iou_threshold=0.3,
                 max_faces=MAX_FACE_NUM):
    """One frame: returns dict(det_index, scores, boxes, keypoints, poses) in NMS order."""
    anc = anchors()
    loc = np.concatenate([np.asarray(loc0, np.float32).reshape(-1, 16), np.asarray(loc1, np.float32).reshape(-1, 16)])
    cls = np.concatenate([np.asarray(cls0, np.float32).ravel(), np.asarray(cls1, np.float32).ravel()])
    thr = score_logit_threshold(score_threshold)
    good = np.where(cls > np.float32(thr))[0]
    scores = (np.float32(1.0) / (np.float32(1.0) + np.exp(-cls[good]))).astype(np.float32)
    boxes = np.zeros((len(good), 4))
    kps = np.zeros((len(good), KEY_POINT_SIZE, 2))
    for k, d in enumerate(good):
        ax, ay = anc[d, 0], anc[d, 1]
        sx, sy, w, h = (float(v) for v in loc[d, :4])
        cx = (sx + ax * INPUT) / INPUT
        cy = (sy + ay * INPUT) / INPUT
        w /= INPUT
        h /= INPUT
        for j in range(KEY_POINT_SIZE):
            kps[k, j] = ((float(loc[d, 4 + 2 * j]) + ax * INPUT) / INPUT,
                         (float(loc[d, 5 + 2 * j]) + ay * INPUT) / INPUT)
        boxes[k] = (cx - w * 0.5, cy - h * 0.5, cx + w * 0.5, cy + h * 0.5)
    sel = non_max_suppression(boxes, scores, max_faces, iou_threshold)
    det = good[sel]
    poses = []
    for d in det:
        if d < 512:
            cell = d // 2
            poses.append(pose_front[cell // 16, cell % 16])
        else:
            cell = (d - 512) // 6
            poses.append(pose_back[cell // 8, cell % 8])
    poses = np.asarray(poses, np.float32).reshape(-1, 3)
    return dict(det_index=det, scores=scores[sel], boxes=boxes[sel], keypoints=kps[sel], poses=poses)


def gather_features(det_index, tap_front, tap_back, k=1):
    """Feature-dataset extraction for one frame — TEST INFRASTRUCTURE.

    For each of the first k kept detections, the regressor input its pose came from: the same cell
    arithmetic as the pose gather at blazeFaceDetectorH5.py:342-353 applied to the tapped maps
    (JoinModels.py:114 taps re_lu_10 -> tap_front (16,16,C0), re_lu_15 -> tap_back (8,8,C1)).
    Returns (feat_front (k,C0), feat_back (k,C1), src (k,) 0 front / 1 back / -1 empty)."""
    c0, c1 = tap_front.shape[-1], tap_back.shape[-1]
    f0 = np.zeros((k, c0), np.float32)
    f1 = np.zeros((k, c1), np.float32)
    src = np.full(k, -1, np.int32)
    for j, d in enumerate(list(det_index)[:k]):
        if d < 512:
            cell = d // 2
            f0[j] = tap_front[cell // 16, cell % 16]
            src[j] = 0
        else:
            cell = (d - 512) // 6
            f1[j] = tap_back[cell // 8, cell % 8]
            src[j] = 1
    return f0, f1, src
