"""mlp2v vs the 12-wave split kernel (HPE_MLP2_V=0 path) vs the exact-fp32 kernel on one training
gradient of create_model(F, act, dropout) — per parameter tensor: max |diff| / max |g| and where
(hidden units, input channels) the 8-wave kernel departs.  argv: F act dropout side n"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'head-pose-estimation-model_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import hpe  # noqa: E402
from hpe import keras, _lib  # noqa: E402
from util import features, labels  # noqa: E402

F, act, dr, side, n = int(sys.argv[1]), sys.argv[2], float(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
P = side * side
hpe.set_seed(F)
keras.backend.clear_session()
reg = keras.regularizers.l2(0.1)
inp = keras.Input(shape=(None, None, 96))
h = keras.layers.Conv2D(F, 1, padding='same', activation=act, kernel_regularizer=reg, bias_regularizer=reg)(inp)
h = keras.layers.SpatialDropout2D(dr)(h)
o = keras.layers.Conv2D(3, 1, padding='same', kernel_regularizer=reg, bias_regularizer=reg)(h)
o = keras.layers.SpatialDropout2D(dr)(o)
m = keras.Model(inp, o)
m.compile(optimizer=keras.optimizers.Adam(learning_rate=2.8e-4), loss='mse')
eng = m._eng()
x = features(n, 96, seed=F + 7, h=side, w=side)
y = labels(n, seed=F + 8)
xt = torch.from_numpy(x.reshape(n * P, 96)).cuda()
yt = torch.from_numpy(y.reshape(n, 3).astype(np.float32)).cuda()
inv = 1.0 / (n * P * 3)
lib = _lib.load()


def grad():
    return eng.gradient(xt, yt, P, None, n, inv, seed=5).cpu().numpy().astype(np.float64).copy()


gv = grad()
os.environ['HPE_MLP2_V'] = '0'
gw = grad()
prev = lib.hpe_set_exact_fp32(1)
ge = grad()
lib.hpe_set_exact_fp32(prev)
os.environ.pop('HPE_MLP2_V')
npt = eng.n_train
scale = np.abs(ge[:npt]).max()
print('launch grid', lib.hpe_launch_grid(eng.program('train', P).h, n * P), 'rows', n * P,
      'v vs exact (params) %.2e' % (np.abs(gv[:npt] - ge[:npt]).max() / scale))
for name, (off, shp) in sorted(eng.layout.param_index.items(), key=lambda kv: kv[1][0]):
    sz = int(np.prod(shp))
    for tag, g in (('v', gv), ('w', gw)):
        d = np.abs(g[off:off + sz] - ge[off:off + sz])
        print('%-18s %s max|d|/max|g| %.2e' % (name, tag, d.max() / scale))
    d = np.abs(gv[off:off + sz] - ge[off:off + sz]).reshape(shp[-2:] if len(shp) >= 2 else shp)
    if d.ndim == 2 and d.max() / scale > 1e-6:
        bad = np.argwhere(d / scale > 1e-6)
        print('   v-bad rows %s ... cols %s ... (%d entries)' % (np.unique(bad[:, 0])[:12].tolist(), np.unique(bad[:, 1])[:24].tolist(), len(bad)))
    elif d.ndim == 1 and d.max() / scale > 1e-6:
        print('   v-bad idx %s (%d)' % (np.nonzero(d / scale > 1e-6)[0][:24].tolist(), int((d / scale > 1e-6).sum())))
print('loss sums v', gv[npt:npt + 2], 'w', gw[npt:npt + 2], 'exact', ge[npt:npt + 2])
