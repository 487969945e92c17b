"""Run the fused training gradient of a checkpoint (default sqnu665j) on side x side maps (default
96: P = 9216; n images) R times in one process and report every run whose result differs from the
first (race screen): prints the differing entries.  argv: n R [rid side]"""
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
rid = sys.argv[3] if len(sys.argv) > 3 else 'sqnu665j'
side = int(sys.argv[4]) if len(sys.argv) > 4 else 96
mc, w = fixture(rid)
eng = Engine(mc, w)
P = side * side
c = int(mc['config']['layers'][0]['config']['batch_input_shape'][-1])
x = features(n, c, seed=21, h=side, w=side)
y = labels(n, seed=22)
xt = torch.from_numpy(x.reshape(n * P, c)).cuda()
yt = torch.from_numpy(y.reshape(n, 3).astype(np.float32)).cuda()
gs = [eng.gradient(xt, yt, P, None, n, 1.0 / (n * P * 3), seed=5).cpu().numpy().copy() for _ in range(R)]
ref = gs[0]
from hpe import _lib  # noqa: E402
lib = _lib.load()
prev = lib.hpe_set_exact_fp32(1)
g_exact = eng.gradient(xt, yt, P, None, n, 1.0 / (n * P * 3), seed=5).cpu().numpy().copy()
lib.hpe_set_exact_fp32(prev)
nbad = 0
for i, g in enumerate(gs[1:], 1):
    d = np.nonzero(g != ref)[0]
    if len(d):
        nbad += 1
        rel = float(np.abs(g - ref).max() / max(np.abs(ref).max(), 1e-30))
        if np.array_equal(g, g_exact) or np.array_equal(ref, g_exact):
            print('run %d: %s equals the exact-fp32 kernel\'s gradient (guard fallback)'
                  % (i, 'this run' if np.array_equal(g, g_exact) else 'run 0'), flush=True)
        print('run %d: %d entries differ (max |diff| / max |g| = %.2e), first %s'
              % (i, len(d), rel, d[:12].tolist()), flush=True)
print('%s side %d n=%d: %d of %d runs differ from run 0' % (rid, side, n, nbad, R - 1), flush=True)
