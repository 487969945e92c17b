"""Dump the fused training gradient of sqnu665j at P = 9216 (2 images) with the library HPE_LIB
points at, for A/B diagnosis of kernel variants: gpurun_out/diag_<tag>.npy"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'head-pose-estimation-model_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
from util import features, fixture, labels  # noqa: E402
from hpe.engine import Engine  # noqa: E402

tag = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 2
mc, w = fixture('sqnu665j')
eng = Engine(mc, w)
P = 96 * 96
x = features(n, 96, seed=21, h=96, w=96)
y = labels(n, seed=22)
xt = torch.from_numpy(x.reshape(n * P, 96)).cuda()
yt = torch.from_numpy(y.reshape(n, 3).astype(np.float32)).cuda()
g = eng.gradient(xt, yt, P, None, n, 1.0 / (n * P * 3), seed=5).cpu().numpy().copy()
np.save(os.path.join(ROOT, 'gpurun_out', 'diag_%s.npy' % tag), g)
print(tag, 'n_train', eng.n_train, 'layout', {k: v for k, v in eng.layout.param_index.items()})
