"""Race screen: run the fused training gradient of a checkpoint (default sqnu665j) on side x side
maps (default 96: P = 9216; n images) R times in one process on identical inputs and report every
run whose result differs from the first: which parameter tensors differ (and, for the first-layer
kernel, which input channels / hidden units), whether the launch's fp16-split guard fired (the
exact-fp32 twin recomputed it) and which check set it (hpe_guard_peek).  argv: n R [rid side]
HPE_SPLIT_ONLY=1 runs the split kernel without its exact twin."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'head-pose-estimation-model_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
from util import features, fixture, labels  # noqa: E402
from hpe.engine import Engine  # noqa: E402
from hpe import _lib  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
R = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rid = sys.argv[3] if len(sys.argv) > 3 else 'sqnu665j'
side = int(sys.argv[4]) if len(sys.argv) > 4 else 96
lib = _lib.load()
print('build', _lib.build_id(), 'split_only', os.environ.get('HPE_SPLIT_ONLY', '0'), flush=True)
mc, w = fixture(rid)
eng = Engine(mc, w)
P = side * side
c = int(mc['config']['layers'][0]['config']['batch_input_shape'][-1])
x = features(n, c, seed=21, h=side, w=side)
y = labels(n, seed=22)
xt = torch.from_numpy(x.reshape(n * P, c)).cuda()
yt = torch.from_numpy(y.reshape(n, 3).astype(np.float32)).cuda()
prog = eng.program('train', P)
peek = (ctypes.c_int32 * 33)()


SLEEP = float(os.environ.get('DIAG_SLEEP', '0'))   # idle the GPU between launches (clock ramp)


def run():
    if SLEEP:
        import time
        time.sleep(SLEEP)
    g = eng.gradient(xt, yt, P, None, n, 1.0 / (n * P * 3), seed=5).cpu().numpy().copy()
    _lib.check(lib.hpe_guard_peek(prog.h, peek), 'hpe_guard_peek')
    ep = peek[0]
    slot = ep % 16
    return g, peek[1 + slot] == ep, peek[17 + slot]


def regions(d):
    out = []
    for name, (o, shp) in sorted(eng.layout.param_index.items(), key=lambda kv: kv[1][0]):
        sz = int(np.prod(shp))
        sel = d[(d >= o) & (d < o + sz)] - o
        if len(sel) == 0:
            continue
        if len(shp) >= 2:
            F = shp[-1]
            rows, cols = np.unique(sel // F), np.unique(sel % F)
            pairs = ' (row, col) %s' % [(int(v // F), int(v % F)) for v in sel] if len(sel) <= 48 else ''
            out.append('%s[%d of %d: rows %s cols %s%s]' % (name, len(sel), sz, rows[:8].tolist(), cols[:12].tolist(), pairs))
        else:
            out.append('%s[%d of %d: %s]' % (name, len(sel), sz, sel[:8].tolist()))
    tail = d[d >= eng.n_train]
    if len(tail):
        out.append('loss sums %s' % (tail - eng.n_train).tolist())
    return ' '.join(out)


runs = [run() for _ in range(R)]
ref, f0, w0 = runs[0]
prev = lib.hpe_set_exact_fp32(1)
g_exact = eng.gradient(xt, yt, P, None, n, 1.0 / (n * P * 3), seed=5).cpu().numpy().copy()
lib.hpe_set_exact_fp32(prev)
nbad = sum(1 for _, f, _ in runs if f)
import hashlib  # noqa: E402
print('guard fired in %d of %d launches (run 0: %s); run-0 gradient sha1 %s'
      % (nbad, R, f0, hashlib.sha1(ref.tobytes()).hexdigest()[:12]), flush=True)
ndiff = 0
for i, (g, fired, why) in enumerate(runs[1:], 1):
    d = np.nonzero(g != ref)[0]
    if fired:
        print('run %d: guard fired (why %d)%s' % (i, why, ', equals the exact kernel' if np.array_equal(g, g_exact) else ''), flush=True)
    if len(d):
        ndiff += 1
        scale = max(np.abs(ref).max(), 1e-30)
        rel = float(np.nanmax(np.abs(g - ref)) / scale)
        print('run %d: %d entries differ (max |diff| / max |g| = %.2e, finite %s, exact-equal %s): %s'
              % (i, len(d), rel, bool(np.isfinite(g).all()), np.array_equal(g, g_exact), regions(d)), flush=True)
print('%s side %d n=%d: %d of %d runs differ from run 0' % (rid, side, n, ndiff, R - 1), flush=True)
save = os.environ.get('DIAG_SAVE')
if save:
    # every distinct gradient of the process (the run-0 reference first) with its run indices
    uniq, who = [], []
    for i, (g, _, _) in enumerate(runs):
        for k, u in enumerate(uniq):
            if np.array_equal(g, u):
                who[k].append(i)
                break
        else:
            uniq.append(g)
            who.append([i])
    if len(uniq) > 1:
        np.savez(save, grads=np.stack(uniq), counts=np.array([len(w) for w in who]),
                 first=np.array([w[0] for w in who]), exact=g_exact)
        print('saved %d distinct gradients to %s' % (len(uniq), save), flush=True)
