"""test_train_step_bounded_matches_unbounded[sqnu665j-64-4] as a diagnostic: the unbounded launch
(split kernel + exact twin) and the bounded one (split only) on identical inputs, repeated; prints
which parameter regions differ and the guard state of each launch."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'head-pose-estimation-model_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
from util import features, fixture, labels, input_channels  # noqa: E402
from hpe.engine import Engine  # noqa: E402
from hpe import _lib  # noqa: E402

rid, P, n, R = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
lib = _lib.load()
print('build', _lib.build_id(), flush=True)
mc, w = fixture(rid)
c = input_channels(mc)
eng = Engine(mc, w)
side = int(round(P ** 0.5))
x = features(n, c, seed=31, h=side, w=side)
y = labels(n, seed=32)
xt = torch.from_numpy(x.reshape(n * P, c)).cuda()
yt = torch.from_numpy(y.reshape(n, 3).astype(np.float32)).cuda()
bound = float(np.abs(x).max())
prog = eng.program('train', P)
print('kind', prog.prog.kind, 'grid', lib.hpe_launch_grid(prog.h, n * P), flush=True)
peek = (ctypes.c_int32 * 33)()


def g(b):
    r = eng.gradient(xt, yt, P, None, n, 1.0 / (n * P * 3), seed=3, x_bound=b).cpu().numpy().copy()
    _lib.check(lib.hpe_guard_peek(prog.h, peek), 'hpe_guard_peek')
    ep = peek[0]
    return r, (peek[1 + ep % 16] == ep, peek[17 + ep % 16])


def where(d):
    out = []
    for name, (o, shp) in sorted(eng.layout.param_index.items(), key=lambda kv: kv[1][0]):
        sz = int(np.prod(shp))
        sel = d[(d >= o) & (d < o + sz)] - o
        if len(sel):
            out.append('%s[%s]' % (name, ','.join(str(int(s)) for s in sel[:20])))
    return ' '.join(out) or ('tail %s' % d[:8])


ref, gr = g(0.0)
print('ref guard', gr, flush=True)
for i in range(R):
    for b in (0.0, bound):
        r, gi = g(b)
        d = np.nonzero(r != ref)[0]
        if len(d) or gi[0]:
            print('run %d bound %g guard %s: %d differ max %.3e %s' % (i, b, gi, len(d),
                  float(np.abs(r - ref).max()), where(d)), flush=True)
print('done', flush=True)
