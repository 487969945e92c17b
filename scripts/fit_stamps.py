"""Phase timing of the whole-epoch kernel (csrc/hpe_fit.hip built with -DFIT_STAMPS into
hpe/libhpe_stamps.so; run with HPE_LIB pointing at it): one fused fit epoch of create_model(360),
P = 1, prints per-phase s_memtime totals of workgroups 0 and G-1."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'head-pose-estimation-model_amd'))
import bench  # noqa: E402
from hpe import keras  # noqa: E402

bs = int(sys.argv[1]) if len(sys.argv) > 1 else 128
n = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
rng = np.random.default_rng(0)
x = np.maximum(0.0, 0.6 * rng.standard_normal((n, 1, 1, 96)) - 0.3).astype(np.float32)
y = (20 * rng.standard_normal((n, 1, 1, 3))).astype(np.float32)
m = bench.build_train_model(keras)
m.fit(x, y, batch_size=bs, epochs=1, verbose=0)
import torch  # noqa: E402
torch.cuda.synchronize()
t0 = time.perf_counter()
m.fit(x, y, batch_size=bs, epochs=1, verbose=0)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
print('fused=%s steps=%d wall %.3f ms -> %.2f us/step' % (m._last_fit_fused, -(-n // bs), dt * 1e3, dt / -(-n // bs) * 1e6))
