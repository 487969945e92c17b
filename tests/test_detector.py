"""Detector post-processing: SSD anchors pinned to the reference's generator,
the oracle's TF-NMS restatement on hand-checkable cases, and (GPU) the batched hpe_detect kernel
against the oracle frame by frame.  Bit-exact bar: counts, kept detection indices (NMS order) and
poses must be identical; fp64 boxes / keypoints equal to 1e-12; fp32 scores to 1 ulp (rtol 2e-7)."""
import os

import numpy as np
import pytest

from oracle import detector_ref as D
from util import GOLDEN, fixture

RID = 'reg1-stoqa9pt-reg2-hrchr82r-selected'


def test_anchors_match_reference_generator():
    g = np.load(os.path.join(GOLDEN, 'anchors_blazeface_128.npy'))
    assert g.shape == (896, 4)
    np.testing.assert_array_equal(D.anchors(), g)


def test_nms_restatement_cases():
    b = np.array([[0, 0, 1, 1], [0, 0, 1, 1], [0.5, 0, 1.5, 1], [2, 2, 3, 3], [0, 0, 1, 1.0]])
    s = np.array([0.9, 0.9, 0.8, 0.7, 0.95], np.float32)
    # 4 (0.95) first; 0 and 1 identical to it -> suppressed; 2 has IoU 1/3 > 0.3 -> suppressed; 3 kept
    assert D.non_max_suppression(b, s, 100, 0.3).tolist() == [4, 3]
    # IoU exactly at the threshold is kept (suppress iff IoU > threshold)
    assert D.non_max_suppression(b[[0, 2]], s[[0, 2]], 100, np.float32(1 / 3)).tolist() == [0, 1]
    # ties go to the lower index; max_output_size caps
    assert D.non_max_suppression(b[[3, 0]], np.array([0.5, 0.5], np.float32), 1, 0.3).tolist() == [0]
    # empty
    assert D.non_max_suppression(np.zeros((0, 4)), np.zeros(0, np.float32), 100, 0.3).size == 0


def synthetic_outputs(n, seed=0):
    """Detector outputs exercising: no candidates, heavy overlap, >max_faces survivors, score ties."""
    rng = np.random.default_rng(seed)
    cls0 = rng.normal(0, 2, (n, 512, 1)).astype(np.float32)
    cls1 = rng.normal(0, 2, (n, 384, 1)).astype(np.float32)
    loc0 = np.zeros((n, 512, 16), np.float32)
    loc1 = np.zeros((n, 384, 16), np.float32)
    loc0[:] = rng.normal(0, 4, loc0.shape)
    loc1[:] = rng.normal(0, 4, loc1.shape)
    loc0[..., 2:4] = rng.uniform(8, 40, (n, 512, 2))
    loc1[..., 2:4] = rng.uniform(8, 40, (n, 384, 2))
    pose0 = rng.normal(0, 20, (n, 16, 16, 3)).astype(np.float32)
    pose1 = rng.normal(0, 20, (n, 8, 8, 3)).astype(np.float32)
    if n > 1:                       # frame 1: nothing above threshold
        cls0[1] = -5
        cls1[1] = -5
    if n > 2:                       # frame 2: tiny boxes on every anchor -> one per cell survives (> 100)
        cls0[2] = 3
        cls1[2] = 3
        loc0[2, :, :4] = [0, 0, 0.5, 0.5]
        loc1[2, :, :4] = [0, 0, 0.5, 0.5]
    if n > 3:                       # frame 3: ties in score
        cls0[3] = np.round(cls0[3])
        cls1[3] = np.round(cls1[3])
    return [cls0, cls1, loc0, loc1, pose0, pose1]


def _check_frame(got, ref, i):
    c = int(got['count'][i])
    assert c == len(ref['det_index']), (i, c, len(ref['det_index']))
    np.testing.assert_array_equal(got['det_index'][i, :c], ref['det_index'])
    np.testing.assert_allclose(got['scores'][i, :c], ref['scores'], rtol=2e-7, atol=0)
    np.testing.assert_allclose(got['boxes'][i, :c], ref['boxes'], rtol=0, atol=1e-12)
    np.testing.assert_allclose(got['keypoints'][i, :c], ref['keypoints'], rtol=0, atol=1e-12)
    np.testing.assert_array_equal(got['poses'][i, :c], ref['poses'])


@pytest.mark.gpu
def test_detect_kernel_matches_oracle():
    import torch
    from hpe import _lib
    from hpe.detector import BlazeFaceDetector
    mc, w = fixture(RID)
    det = BlazeFaceDetector(mc, w)
    n = 6
    outs = synthetic_outputs(n, seed=3)
    dev = [torch.from_numpy(o).cuda() for o in outs]
    r = det.postprocess(dev)
    got = {k: v.cpu().numpy() for k, v in r.items()}
    assert int(got['count'][1]) == 0 and int(got['count'][2]) == D.MAX_FACE_NUM
    for i in range(n):
        ref = D.detect_frame(outs[0][i], outs[1][i], outs[2][i], outs[3][i], outs[4][i], outs[5][i])
        _check_frame(got, ref, i)
    assert _lib.load() is not None


@pytest.mark.gpu
def test_detector_end_to_end_on_network_outputs():
    """detect_batch == oracle post-processing applied to the same frames' network outputs."""
    import torch
    from hpe.detector import BlazeFaceDetector
    mc, w = fixture(RID)
    det = BlazeFaceDetector(mc, w, scoreThreshold=0.4, iouThreshold=0.3)
    frames = np.random.default_rng(11).uniform(-1, 1, (4, 128, 128, 3)).astype(np.float32)
    res = det.detect_batch(frames)
    outs = [o.cpu().numpy() for o in det.net.forward(torch.from_numpy(frames).cuda())]
    for i in range(4):
        ref = D.detect_frame(*(o[i] for o in outs))
        assert len(res[i].scores) == len(ref['scores'])
        np.testing.assert_allclose(res[i].boxes, ref['boxes'], rtol=0, atol=1e-12)
        np.testing.assert_array_equal(res[i].poses, ref['poses'])
