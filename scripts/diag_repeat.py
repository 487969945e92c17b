"""Run the fused training gradient of sqnu665j at P = 9216 (n images) R times in one process and
report every run whose result differs from the first (race hunting): prints the differing entries"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'head-pose-estimation-model_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
from util import features, fixture, labels  # noqa: E402
from hpe.engine import Engine  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
R = int(sys.argv[2]) if len(sys.argv) > 2 else 20
mc, w = fixture('sqnu665j')
eng = Engine(mc, w)
P = 96 * 96
x = features(n, 96, seed=21, h=96, w=96)
y = labels(n, seed=22)
xt = torch.from_numpy(x.reshape(n * P, 96)).cuda()
yt = torch.from_numpy(y.reshape(n, 3).astype(np.float32)).cuda()
gs = [eng.gradient(xt, yt, P, None, n, 1.0 / (n * P * 3), seed=5).cpu().numpy().copy() for _ in range(R)]
ref = gs[0]
nbad = 0
for i, g in enumerate(gs[1:], 1):
    d = np.nonzero(g != ref)[0]
    if len(d):
        nbad += 1
        print('run %d: %d entries differ, first %s' % (i, len(d), d[:12].tolist()), flush=True)
print('n=%d: %d of %d runs differ from run 0' % (n, nbad, R - 1), flush=True)
