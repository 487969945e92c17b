"""Feature-dataset extraction: hpe.features.FeatureExtractor and the
hpe_gather_features kernel.

Pinning: the reference holds no images and its extractor is outside the repo, so the datasets'
bytes cannot be regenerated here (parity of the rows themselves is unpinned).  What is pinned is the
semantics that ties a feature row to the reference: the row of a detection is the tap vector the
unified model's regressor turned into that detection's pose (blazeFaceDetectorH5.py:342-353,
JoinModels.py:114).  CPU: the oracle's gather fed to the embedded regressors (the reference's own
stoqa9pt / hrchr82r weights) reproduces the oracle's detector poses exactly.  GPU: the kernel's rows
are bit-identical to the device taps at the oracle-selected cells, within the BlazeFace tolerance of
the oracle's taps, and predicting on them reproduces the detector's poses.

Random frames score far below the reference's 0.7 (max sigmoid ~0.3), so the tests run the same
pipeline at score threshold 0.15 and up to 8 faces per frame (both anchor sets represented)."""
import numpy as np
import pytest

from oracle import detector_ref as D
from oracle import keras_ref as K
from util import fixture

RID = 'reg1-stoqa9pt-reg2-hrchr82r-selected'
THR, KF = 0.15, 8
BF_RTOL, BF_ATOL = 1e-4, 1e-3


def _frames(n, seed):
    return np.random.default_rng(seed).uniform(-1, 1, (n, 128, 128, 3)).astype(np.float32)


def _oracle_with_taps(x):
    mc, w = fixture(RID)
    cfg = dict(mc['config'])
    cfg['output_layers'] = list(cfg['output_layers']) + [['re_lu_10', 0, 0], ['re_lu_15', 0, 0]]
    return [o.detach().numpy() for o in K.Graph(dict(mc, config=cfg), w).forward(x)]


def test_oracle_feature_rows_are_the_regressor_inputs_of_the_poses():
    x = _frames(3, seed=4)
    outs = _oracle_with_taps(x)
    reg = {c: K.Graph(*fixture(r)) for c, r in ((88, 'stoqa9pt'), (96, 'hrchr82r'))}
    seen = set()
    for i in range(len(x)):
        ref = D.detect_frame(*(o[i] for o in outs[:6]), score_threshold=THR, iou_threshold=0.3)
        f0, f1, src = D.gather_features(ref['det_index'], outs[6][i], outs[7][i], k=KF)
        c = min(KF, len(ref['det_index']))
        assert (src[:c] >= 0).all() and (src[c:] == -1).all()
        for j in range(c):
            seen.add(int(src[j]))
            f, ch = (f0[j], 88) if src[j] == 0 else (f1[j], 96)
            assert not (f1[j] if src[j] == 0 else f0[j]).any()
            pose = reg[ch].forward(f.reshape(1, 1, 1, ch)).detach().numpy().reshape(3)
            # the unified graph applied the same weights to the same vector inside the map
            np.testing.assert_allclose(pose, ref['poses'][j], rtol=1e-6, atol=1e-5)
    assert seen == {0, 1}


def test_gather_features_rejects_bad_arguments():
    import ctypes
    from hpe import _lib
    lib = _lib.load()
    z = ctypes.c_void_p(8)
    assert lib.hpe_gather_features(None, z, 1, 1, 1, z, 88, z, 96, z, z, z, None) == 1
    assert lib.hpe_gather_features(z, z, 1, 1, 2, z, 88, z, 96, z, z, z, None) == 1   # k > max_faces
    assert lib.hpe_gather_features(z, z, 1, 1, 1, z, 90, z, 96, z, z, z, None) == 1   # c0 % 4
    assert b'multiples of 4' in lib.hpe_last_error()


@pytest.mark.gpu
def test_gpu_feature_rows_match_taps_and_oracle():
    import torch
    from hpe.features import FeatureExtractor
    mc, w = fixture(RID)
    fe = FeatureExtractor(mc, w, scoreThreshold=THR, max_faces=KF)
    x = _frames(5, seed=6)
    r = fe.extract_device(torch.from_numpy(x).cuda())
    taps = {k: v.cpu().numpy() for k, v in fe.det.net.taps.items()}
    count = r['count'].cpu().numpy()
    det = r['det_index'].cpu().numpy()
    f0, f1, src = (r[k].cpu().numpy() for k in ('feat88', 'feat96', 'src'))
    outs = _oracle_with_taps(x)
    seen = set()
    for i in range(len(x)):
        c = int(count[i])
        # bit-exact gather from the device taps at the kernel's own detections
        e0, e1, es = D.gather_features(det[i, :c], taps['re_lu_10'][i], taps['re_lu_15'][i], k=KF)
        np.testing.assert_array_equal(src[i], es)
        np.testing.assert_array_equal(f0[i], e0)
        np.testing.assert_array_equal(f1[i], e1)
        seen |= set(es[es >= 0].tolist())
        # and the oracle's detections / rows
        ref = D.detect_frame(*(o[i] for o in outs[:6]), score_threshold=THR, iou_threshold=0.3)
        np.testing.assert_array_equal(det[i, :c], ref['det_index'])
        o0, o1, _ = D.gather_features(ref['det_index'], outs[6][i], outs[7][i], k=KF)
        np.testing.assert_allclose(f0[i], o0, rtol=BF_RTOL, atol=BF_ATOL)
        np.testing.assert_allclose(f1[i], o1, rtol=BF_RTOL, atol=BF_ATOL)
    assert seen == {0, 1}


@pytest.mark.gpu
def test_gpu_build_datasets_and_predict_reproduces_detector_poses(tmp_path):
    """The written .npz files load with the reference's loader contract and a regressor predicting
    on them returns the poses the detector reported for the same detections."""
    import hpe
    from hpe.features import FeatureExtractor
    mc, w = fixture(RID)
    fe = FeatureExtractor(mc, w, scoreThreshold=THR, max_faces=KF)
    x = _frames(7, seed=8)
    poses = np.random.default_rng(1).normal(0, 20, (7, 3))
    p88, p96 = fe.build_datasets(x, poses, str(tmp_path / 'SYN'))
    assert p88.endswith('SYN_features_88_0.15_8.npz') and p96.endswith('SYN_features_96_0.15_8.npz')
    d88, d96 = np.load(p88), np.load(p96)
    assert d88['features'].dtype == np.float32 and d88['poses'].dtype == np.float64
    assert d88['features'].shape[1] == 88 and d96['features'].shape[1] == 96
    res = fe.det.detect_batch(x)
    n_det = sum(min(KF, len(r.scores)) for r in res)
    assert len(d88['features']) + len(d96['features']) == n_det
    # per-detection poses from the detector, split by anchor set in frame / NMS order
    f0, i0, f1, i1 = fe.extract(x)
    np.testing.assert_array_equal(d88['poses'], poses[i0])
    np.testing.assert_array_equal(d96['poses'], poses[i1])
    r = fe.extract_device(x)
    src, det, pz = r['src'].cpu().numpy(), r['det_index'].cpu().numpy(), r['poses'].cpu().numpy()
    want0 = np.array([pz[i, j] for i in range(7) for j in range(KF) if src[i, j] == 0]).reshape(-1, 3)
    want1 = np.array([pz[i, j] for i in range(7) for j in range(KF) if src[i, j] == 1]).reshape(-1, 3)
    m88 = hpe.load_model(__import__('util').MODELS + '/stoqa9pt')
    m96 = hpe.load_model(__import__('util').MODELS + '/hrchr82r')
    np.testing.assert_allclose(m88.predict(d88['features'].reshape(-1, 1, 1, 88)).reshape(-1, 3), want0,
                               rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(m96.predict(d96['features'].reshape(-1, 1, 1, 96)).reshape(-1, 3), want1,
                               rtol=1e-5, atol=1e-4)
