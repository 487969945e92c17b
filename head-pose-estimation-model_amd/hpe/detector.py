"""Batched face detection + head pose: the unified BlazeFace graph (hpe.blazeface) followed by the
detector post-processing kernel (csrc/hpe_detect.hip, C ABI ``hpe_detect``).

Mirrors ``blazeFaceDetector`` of BlazePoser/blazeFaceDetectorH5.py:80-364 for frames that are
already preprocessed to the model input (``prepareInputForInference``, :244-269: RGB, /255, bicubic
resize to 128x128, (x - 0.5) / 0.5 — done by the caller; cv2 / the webcam loop are out of scope):
``detectFaces(frame)`` for one frame and ``detect_batch(frames)`` for a batch, returning
``Results(boxes, keypoints, scores, poses)`` per frame (:359-364).
"""
import ctypes
import math

import numpy as np
import torch

from . import _lib
from .blazeface import BlazeFace

KEY_POINT_SIZE = 6      # blazeFaceDetectorH5.py:8
MAX_FACE_NUM = 100      # blazeFaceDetectorH5.py:9


class Results:
    def __init__(self, boxes, keypoints, scores, poses):
        self.boxes = boxes
        self.keypoints = keypoints
        self.scores = scores
        self.poses = poses


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


class BlazeFaceDetector:
    def __init__(self, model_config, weights, scoreThreshold=0.4, iouThreshold=0.3, device=None,
                 max_faces=MAX_FACE_NUM):
        self.scoreThreshold = scoreThreshold
        self.iouThreshold = iouThreshold
        self.sigmoidScoreThreshold = math.log(scoreThreshold / (1 - scoreThreshold))
        self.max_faces = int(max_faces)
        self.net = BlazeFace(model_config, weights, device=device)
        self.device = self.net.device
        shp = self.net.output_shapes(1)
        outs = self.net.structure['outputs']
        want = [(1, 512, 1), (1, 384, 1), (1, 512, 16), (1, 384, 16), (1, 16, 16, 3), (1, 8, 8, 3)]
        if [shp[o] for o in outs] != want:
            raise ValueError('unified model outputs %s do not match the BlazeFace front detector %s'
                             % ([shp[o] for o in outs], want))

    def postprocess(self, outs):
        """outs: the six device outputs of the unified graph -> device result tensors."""
        n = outs[0].shape[0]
        M = self.max_faces
        dev = self.device
        count = torch.zeros(n, dtype=torch.int32, device=dev)
        det = torch.empty((n, M), dtype=torch.int32, device=dev)
        scores = torch.empty((n, M), dtype=torch.float32, device=dev)
        boxes = torch.empty((n, M, 4), dtype=torch.float64, device=dev)
        kps = torch.empty((n, M, KEY_POINT_SIZE, 2), dtype=torch.float64, device=dev)
        poses = torch.empty((n, M, 3), dtype=torch.float32, device=dev)
        lib = _lib.load()
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        o = [x.contiguous() for x in outs]
        _lib.check(lib.hpe_detect(_ptr(o[0]), _ptr(o[1]), _ptr(o[2]), _ptr(o[3]), _ptr(o[4]), _ptr(o[5]), n,
                                  float(np.float32(self.sigmoidScoreThreshold)), float(self.iouThreshold), M,
                                  _ptr(count), _ptr(det), _ptr(scores), _ptr(boxes), _ptr(kps), _ptr(poses),
                                  stream), 'hpe_detect')
        return dict(count=count, det_index=det, scores=scores, boxes=boxes, keypoints=kps, poses=poses)

    def detect_batch(self, frames):
        """frames: (n, 128, 128, 3) preprocessed input (numpy or device tensor) -> [Results] * n."""
        x = frames if torch.is_tensor(frames) else torch.from_numpy(np.ascontiguousarray(frames, np.float32))
        x = x.to(self.device, torch.float32)
        r = self.postprocess(self.net.forward(x))
        h = {k: v.cpu().numpy() for k, v in r.items()}
        res = []
        for i in range(x.shape[0]):
            c = int(h['count'][i])
            res.append(Results(h['boxes'][i, :c], h['keypoints'][i, :c], h['scores'][i, :c],
                               h['poses'][i, :c] if c else np.zeros((0, 3), np.float32)))
        return res

    def detectFaces(self, frame):
        f = np.asarray(frame, np.float32)
        if f.ndim == 3:
            f = f[None]
        return self.detect_batch(f)[0]
