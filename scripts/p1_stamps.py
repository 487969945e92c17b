"""Phase stamps of the 12-wave mlp2_kernel in the P = 1 per-step path (Model-96 create_model(360),
batch 128 / 512): run with HPE_LIB=varlibs/libhpe_stamps.so (hpe_mlp2.o built with -DMLP2_STAMPS);
the kernel's device printf lines go to stdout, summarised by scripts/p1_stamps_sum.py."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))
os.environ['HPE_FIT_FUSED'] = '0'
import bench  # noqa: E402
from hpe import keras  # noqa: E402

bs = int(sys.argv[1]) if len(sys.argv) > 1 else 128
rng = np.random.default_rng(0)
n = bs * 40
x = np.maximum(0.0, 0.6 * rng.standard_normal((n, 1, 1, 96)) - 0.3).astype(np.float32)
y = (20 * rng.standard_normal((n, 1, 1, 3))).astype(np.float32)
m = bench.build_train_model(keras)
m.fit(x, y, batch_size=bs, epochs=2, verbose=0)
print('DONE', bs, flush=True)
