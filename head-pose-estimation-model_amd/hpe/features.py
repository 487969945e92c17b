"""Feature-dataset extraction on the GPU: regenerate the
``FeatureMaps-Datasets/<set>_features_88_<t>_<k>.npz`` / ``..._96_<t>_<k>.npz`` files the regressors
train on (Model-96/train_96.py:123-130, Model-88/train_88.py:270-280 load them with
``utilities.load_dataset``: keys ``features`` (N, C) float32 and ``poses`` (N, 3) float64).

The extractor itself is outside the reference repo; its interface is pinned by the reference's
files: JoinModels.py:114-116 taps ``re_lu_10`` (16x16x88) and ``re_lu_15`` (8x8x96) of the BlazeFace
front model, and the unified detector reads each detection's pose from the regressor cell of that
detection (BlazePoser/blazeFaceDetectorH5.py:342-353: front anchors d < 512 -> re_lu_10 cell d//2,
back anchors -> re_lu_15 cell (d-512)//6).  A face's feature row is therefore the tap vector the
unified model's regressor consumed for that detection: front detections go to the 88-channel set,
back detections to the 96-channel set, ``<t>`` is the detector score threshold (0.7) and ``<k>`` the
number of faces kept per frame (1).  This is what the dataset sizes show (AFLW2000: 9 rows in the
_88 set + 1809 in the _96 set of 2000 frames).

Pipeline, all on the device: hpe_blazeface_forward (taps written once, in HBM) -> hpe_forward of
the two embedded regressors -> hpe_detect (threshold, decode, NMS) -> hpe_gather_features.  Frames
must already be the model input (``prepareInputForInference``, blazeFaceDetectorH5.py:244-269:
bicubic resize to 128x128 and (x/255 - 0.5)/0.5 are the caller's; the image decoders, cv2 and
tf.image are not part of this image).
"""
import ctypes
import os

import numpy as np
import torch

from . import _lib
from .detector import BlazeFaceDetector


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


class FeatureExtractor:
    """``extract(frames)`` -> per-frame device features of the first ``max_faces`` detections;
    ``build_datasets(frames, poses, prefix)`` -> the two .npz files."""

    def __init__(self, model_config, weights, scoreThreshold=0.7, iouThreshold=0.3, max_faces=1,
                 device=None):
        self.det = BlazeFaceDetector(model_config, weights, scoreThreshold=scoreThreshold,
                                     iouThreshold=iouThreshold, device=device, max_faces=max_faces)
        self.scoreThreshold = scoreThreshold
        self.max_faces = int(max_faces)
        net = self.det.net
        st = net.structure
        # the detector's geometry: the taps feeding the 16x16 and the 8x8 pose maps
        by_shape = {}
        for r in st['regressors']:
            th, tw, c = st['shapes'][r['tap']]
            by_shape[(th, tw)] = (r['tap'], c)
        if (16, 16) not in by_shape or (8, 8) not in by_shape:
            raise ValueError('unified model needs regressors on a 16x16 and an 8x8 tap')
        self.tap_front, self.c_front = by_shape[(16, 16)]
        self.tap_back, self.c_back = by_shape[(8, 8)]
        if self.c_front % 4 or self.c_back % 4:
            raise ValueError('tap channels must be multiples of 4')

    @classmethod
    def from_file(cls, path, **kw):
        from .model import load_model
        m = load_model(path, compile=False)
        return cls(m.model_config, m.weights_dict(), **kw)

    def extract_device(self, frames):
        """frames (n,128,128,3) on the device -> dict of device tensors: feat88 (n,k,C0),
        feat96 (n,k,C1), src (n,k) int32 (0 front / 1 back / -1 none), plus the detector outputs."""
        net, dev = self.det.net, self.det.device
        x = frames if torch.is_tensor(frames) else torch.from_numpy(np.ascontiguousarray(frames, np.float32))
        x = x.to(dev, torch.float32).contiguous()
        n = x.shape[0]
        r = self.det.postprocess(net.forward(x))
        k = self.max_faces
        f0 = torch.empty((n, k, self.c_front), dtype=torch.float32, device=dev)
        f1 = torch.empty((n, k, self.c_back), dtype=torch.float32, device=dev)
        src = torch.empty((n, k), dtype=torch.int32, device=dev)
        t0 = net.taps[self.tap_front].contiguous()
        t1 = net.taps[self.tap_back].contiguous()
        lib = _lib.load()
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        _lib.check(lib.hpe_gather_features(_ptr(r['count']), _ptr(r['det_index']), n, self.max_faces, k,
                                           _ptr(t0), self.c_front, _ptr(t1), self.c_back, _ptr(f0), _ptr(f1),
                                           _ptr(src), stream), 'hpe_gather_features')
        r.update(feat88=f0, feat96=f1, src=src)
        return r

    def extract(self, frames, batch_size=1024):
        """Host arrays: (features_front (m0,C0), frame index (m0,), features_back (m1,C1), frame
        index (m1,)) in frame order, detections in NMS order within a frame."""
        fr, ir, bk, ib = [], [], [], []
        n = len(frames)
        for s in range(0, n, batch_size):
            r = self.extract_device(frames[s:s + batch_size])
            src = r['src'].cpu().numpy()
            f0 = r['feat88'].cpu().numpy()
            f1 = r['feat96'].cpu().numpy()
            i0, j0 = np.nonzero(src == 0)
            i1, j1 = np.nonzero(src == 1)
            fr.append(f0[i0, j0])
            ir.append(i0 + s)
            bk.append(f1[i1, j1])
            ib.append(i1 + s)
        cat = lambda a, c, dt: np.concatenate(a) if a else np.zeros((0,) + c, dt)  # noqa: E731
        return (cat(fr, (self.c_front,), np.float32), cat(ir, (), np.int64),
                cat(bk, (self.c_back,), np.float32), cat(ib, (), np.int64))

    def dataset_names(self, prefix):
        t = ('%g' % self.scoreThreshold)
        return ('%s_features_%d_%s_%d.npz' % (prefix, self.c_front, t, self.max_faces),
                '%s_features_%d_%s_%d.npz' % (prefix, self.c_back, t, self.max_faces))

    def build_datasets(self, frames, poses, prefix, batch_size=1024):
        """Write <prefix>_features_88_<t>_<k>.npz and <prefix>_features_96_<t>_<k>.npz (keys
        ``features`` float32, ``poses`` float64 yaw/pitch/roll of the frame); returns the paths."""
        poses = np.asarray(poses, np.float64).reshape(-1, 3)
        if len(poses) != len(frames):
            raise ValueError('need one (yaw, pitch, roll) per frame: %d frames, %d poses'
                             % (len(frames), len(poses)))
        f0, i0, f1, i1 = self.extract(frames, batch_size)
        p0, p1 = self.dataset_names(prefix)
        d = os.path.dirname(p0)
        if d:
            os.makedirs(d, exist_ok=True)
        np.savez(p0, features=f0, poses=poses[i0])
        np.savez(p1, features=f1, poses=poses[i1])
        return p0, p1
