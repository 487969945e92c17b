"""Time train_88.py's default graph (create_model_complex) in the reference's regime: Model.fit,
batch 128, legacy SGD, on BIWI_Train_Enlarged_features_88 (80/20 split, validation each epoch);
per-step launches (HPE_FIT_FUSED=0) and the whole-epoch kernel (=1).  Prints us/step from the epoch
wall times and, for the fused path, the epoch kernel's own time from HIP events (hpe_kernel_timing).
argv: [epochs] [batch]"""
import ctypes
import importlib.util
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'head-pose-estimation-model_amd'))
import hpe  # noqa: E402
from hpe import _lib, keras  # noqa: E402
from hpe.data import train_test_split  # noqa: E402

epochs = int(sys.argv[1]) if len(sys.argv) > 1 else 6
bs = int(sys.argv[2]) if len(sys.argv) > 2 else 128
d = np.load(os.path.join(ROOT, 'tests', 'golden', 'data', 'BIWI_Train_Enlarged_features_88_0.7_1.npz'))
x = d['features'].reshape(-1, 1, 1, 88).astype(np.float32)
y = d['poses'].reshape(-1, 1, 1, 3).astype(np.float32)
tx, vx, ty, vy = train_test_split(x, y, test_size=0.2, random_state=42)
spec = importlib.util.spec_from_file_location(
    'am88', os.path.join(ROOT, 'head-pose-estimation-model_amd', 'Model-88', 'attention_model.py'))
mod = importlib.util.module_from_spec(spec)
spec.loader.exec_module(mod)
steps = -(-tx.shape[0] // bs)
torch.zeros(1, device='cuda')   # the HIP runtime through torch first, as every other entry point
lib = _lib.load()
print('build', _lib.build_id(), flush=True)
for mode in ('0', '1'):
    os.environ['HPE_FIT_FUSED'] = mode
    keras.backend.clear_session()
    hpe.set_seed(42)
    m = mod.create_model_complex(1e-6, 1e-4)
    m.compile(optimizer=keras.optimizers.SGD(learning_rate=2.8e-4), loss='mse', metrics=['mae'])
    m.fit(tx, ty, batch_size=bs, epochs=1, validation_data=(vx, vy), verbose=0)   # warm-up
    _lib.check(lib.hpe_kernel_timing(4096), 'timing')
    t0 = time.perf_counter()
    m.fit(tx, ty, batch_size=bs, epochs=epochs, validation_data=(vx, vy), verbose=0)
    dt = time.perf_counter() - t0
    buf = (ctypes.c_float * 4096)()
    k = lib.hpe_kernel_times(buf, 4096)
    lib.hpe_kernel_timing(0)
    ms = np.array(buf[:k])
    print('fused=%s batch %d: %.2f us/step (fit wall, validation included), %d timed launches, '
          'longest %s ms, sum %.3f ms per epoch' % (mode, bs, dt / (epochs * steps) * 1e6, k,
                                                    np.round(np.sort(ms)[-3:], 4), ms.sum() / epochs), flush=True)
    if mode == '1':
        big = np.sort(ms)[-epochs:]
        print('  epoch kernel: %.2f us/step' % (big.mean() * 1e3 / steps), flush=True)
    else:
        print('  per-step train kernel: %.2f us (median of %d)' % (np.median(ms) * 1e3, k), flush=True)
