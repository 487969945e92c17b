"""Phase stamps of mlp2r_kernel (csrc/hpe_mlp2.hip, built with -DMLP2R_STAMPS): one Model-88 train88
gradient launch (512 images of 88x88x88); run with HPE_LIB=varlibs/libhpe_rstamps.so."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
import torch  # noqa: E402

import bench  # noqa: E402
from hpe import keras  # noqa: E402

keras.backend.clear_session()
inp = keras.Input(shape=(None, None, 88))
h = keras.layers.Conv2D(64, 1, activation='softsign')(inp)
h = keras.layers.SpatialDropout2D(1e-4)(h)
o = keras.layers.Conv2D(3, 1)(h)
o = keras.layers.SpatialDropout2D(1e-4)(o)
m = keras.Model(inp, o)
m.compile(optimizer=keras.optimizers.Adam(learning_rate=2.8e-4), loss='mse', metrics=['mae'])
eng = m._eng()
n, P = 512, 88 * 88
x, y = bench.synth(n, 88, torch.device('cuda'), P=P, c=88)
for _ in range(2):
    eng.gradient(x, y, P, None, n, 1.0 / (n * P * 3), seed=1)
torch.cuda.synchronize()
print('DONE', flush=True)
