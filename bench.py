"""Benchmark: images/sec of the head-pose regressor training step on 96x96 feature maps.

Workload (BASELINE.json configs[3] restated per GPU): the Model-96
``create_model(num_filters=360, dropout 0, l2 0.1)`` graph of Model-96/train_96.py:65-110 with the
legacy Adam optimizer (lr 2.8e-4), synthetic 96x96x96 feature maps (rows of 96 channels, 9216
positions per image, max(0, 0.6 N(0,1) - 0.3)), labels (yaw, pitch, roll) ~ 20 N(0,1) per image,
512 images per GPU per step (weak scaling: global batch 512 x N).  One step = the fused
forward+loss+backward kernel, the workgroup-partial reduce, one RCCL all-reduce of the flat
gradient when N > 1, and the fused Adam kernel — exactly one ``fit`` step of the reference.
Inputs are resident in HBM before the timed region.

Also reported: ``infer`` (configs[1]: the selected Model-96 head hrchr82r, batch 256 on 96x96
maps, forward only) and ``cpu_baseline`` (the oracle's torch-CPU fp32 restatement of the same
training step on a bounded sample, rank 0, N=1 only).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]   (N>1: torchrun, one rank per GPU)
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'head-pose-estimation-model_amd'))

METRIC = 'images/sec (train+infer) on 96×96 feature maps; yaw/pitch/roll MAE vs ref'
F = 360
H = W = 96
C = 96
PER_GPU = 512
INFER_B = 256
PEAK_FP32 = 157.3e12      # MI355X dense FP32 (vector = matrix), MI355X_MICROARCH.md
PEAK_F16 = 2.5e15         # MI355X dense FP16 MFMA (no sparsity), MI355X_MICROARCH.md
PEAK_HBM = 8.0e12


def gemm_peak():
    """The MFMA ceiling of the regressor GEMMs as libhpe.so runs them: by default every fp32 product is
    three fp16 MFMA products (hi/lo split, fp32 accumulate; csrc/hpe_common.h mfma3), so the
    fp32-equivalent ceiling is the dense fp16 peak / 3; HPE_EXACT_FP32=1 selects the exact fp32 MFMA."""
    if os.environ.get('HPE_EXACT_FP32') == '1':
        return PEAK_FP32, 'exact fp32 MFMA (v_mfma_f32_32x32x2_f32), peak = dense fp32'
    return PEAK_F16 / 3, ('fp32 GEMMs as 3 fp16 MFMA products (hi/lo split, fp32 accumulate); '
                          'peak = 2.5 PFLOP/s dense fp16 / 3, in fp32-equivalent FLOP/s')
# algorithmic work per position: 2*MAC of conv layers only
TRAIN_FLOP_POS = 2 * (C * F + F * 3) * 2 + 2 * F * 3      # fwd + dW + dX(layer 2) = 144,720
INFER_FLOP_POS = 2 * (96 * 32 + 32 * 16 + 16 * 3)         # hrchr82r: 7,264
INFER_BYTES_POS = 4 * 96 + 4 * 3                          # fp32 in + fp32 out


def build_train_model(hpe, keras):
    """create_model() of Model-96/train_96.py:65-110 with num_filters=360, dropout 0, l2 0.1."""
    reg = keras.regularizers.l2(0.1)
    inp = keras.Input(shape=(None, None, 96))
    x1 = keras.layers.Conv2D(filters=F, kernel_size=1, padding='same', activation='tanh',
                             kernel_initializer=keras.initializers.GlorotUniform(),
                             bias_regularizer=reg, kernel_regularizer=reg)(inp)
    x1 = keras.layers.SpatialDropout2D(0.0)(x1)
    out = keras.layers.Conv2D(filters=3, kernel_size=1, padding='same', activation=None,
                              kernel_initializer=keras.initializers.GlorotUniform(),
                              bias_regularizer=reg, kernel_regularizer=reg)(x1)
    out = keras.layers.SpatialDropout2D(0.0)(out)
    m = keras.Model(inputs=inp, outputs=out)
    m.compile(optimizer=keras.optimizers.Adam(learning_rate=0.00028), loss='mse', metrics=['mae'])
    return m


def synth(n_img, seed, device):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    x = torch.randn((n_img * H * W, C), generator=g, device=device, dtype=torch.float32)
    x = torch.clamp_min(0.6 * x - 0.3, 0.0)
    y = 20.0 * torch.randn((n_img, 3), generator=g, device=device, dtype=torch.float32)
    return x.contiguous(), y.contiguous()


def cpu_baseline(weights_cfg, steps_budget_s=12.0):
    """Oracle (torch-CPU fp32 restatement of Keras semantics) timed on a bounded sample:
    training steps on 2 images of 96x96 (18,432 rows) each, legacy Adam, as many as fit in
    ~steps_budget_s."""
    sys.path.insert(0, ROOT)
    from oracle import keras_ref as K
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    mc, w = weights_cfg
    g = K.Graph(mc, w, dtype=torch.float32)
    opt = K.LegacyOptimizer('adam', 2.8e-4)
    rng = np.random.default_rng(0)
    n = 2
    x = np.maximum(0.0, 0.6 * rng.standard_normal((n, H, W, C)) - 0.3).astype(np.float32)
    y = (20 * rng.standard_normal((n, 3))).astype(np.float32)
    xt, yt = torch.from_numpy(x), torch.from_numpy(y)
    K.train_step(g, opt, xt, yt)  # warm-up
    t0 = time.perf_counter()
    steps = 0
    while time.perf_counter() - t0 < steps_budget_s or steps < 2:
        K.train_step(g, opt, xt, yt)
        steps += 1
    dt = time.perf_counter() - t0
    return {'value': steps * n / dt, 'unit': 'images/sec', 'cores': threads, 'kind': 'port',
            'sample': '%d training steps x %d images of 96x96x96 (create_model(360), Adam, '
                      'torch-CPU fp32 restatement, oracle/keras_ref.py), %.1f s' % (steps, n, dt),
            'cpu': _cpu_name()}


def bench_train88(hpe, keras, dev, steps, warmup):
    """Model-88 training on synthetic 88x88 maps (north_star's 88x88 line; configs[2] topology): the
    train_88.py create_model graph (88 -> 64 softsign -> SpatialDropout(1e-4) -> 3 -> SpatialDropout,
    L2 1e-6 on kernels, train_88.py:66-140), legacy Adam lr 2.8e-4, 512 images of 88x88x88 per step."""
    keras.backend.clear_session()
    reg = keras.regularizers.l2(1e-6)
    inp = keras.Input(shape=(None, None, 88))
    x0 = keras.layers.Conv2D(64, 1, padding='same', activation='softsign', kernel_regularizer=reg,
                             kernel_initializer=keras.initializers.GlorotUniform())(inp)
    x0 = keras.layers.SpatialDropout2D(1e-4)(x0)
    x1 = keras.layers.Conv2D(3, 1, padding='same', activation='linear', kernel_regularizer=reg,
                             kernel_initializer=keras.initializers.GlorotUniform())(x0)
    x1 = keras.layers.SpatialDropout2D(1e-4)(x1)
    m = keras.Model(inputs=inp, outputs=x1)
    m.compile(optimizer=keras.optimizers.Adam(learning_rate=0.00028), loss='mse', metrics=['mae'])
    eng = m._eng()
    n, Pm = PER_GPU, 88 * 88
    g = torch.Generator(device=dev)
    g.manual_seed(88)
    x = torch.clamp_min(0.6 * torch.randn((n * Pm, 88), generator=g, device=dev) - 0.3, 0.0).contiguous()
    y = (20.0 * torch.randn((n, 3), generator=g, device=dev)).contiguous()
    inv = 1.0 / (n * Pm * 3)
    stats = torch.zeros((steps + warmup + 1, 2 + eng.optim_grid()), device=dev)
    for i in range(warmup):
        eng.gradient(x, y, Pm, None, n, inv, seed=i + 1)
        eng.optimizer_step(m.optimizer, stats[i])
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    ks = []
    t0 = time.perf_counter()
    for i in range(steps):
        a0 = torch.cuda.Event(enable_timing=True)
        a1 = torch.cuda.Event(enable_timing=True)
        a0.record()
        eng.gradient(x, y, Pm, None, n, inv, seed=warmup + i + 1)
        a1.record()
        ks.append((a0, a1))
        eng.optimizer_step(m.optimizer, stats[warmup + i])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    kms = float(np.mean([a.elapsed_time(b) for a, b in ks]))
    flop = 2 * (88 * 64 + 64 * 3) * 2 + 2 * 64 * 3            # fwd + dW + dX(layer 2) per position
    ach = flop * n * Pm / (kms * 1e-3)
    return {'workload': 'Model-88 create_model (88-64 softsign-3, dropout 1e-4, l2 1e-6) training, legacy Adam, '
                        '512 images of 88x88 feature maps',
            'value': n / dt, 'unit': 'images/sec', 'ms_per_step': dt * 1e3, 'dtype': 'fp32',
            'kernel': eng.program('train', Pm).prog.kind + '_kernel + reduce_kernel',
            'roofline': {'bound': 'mfma', 'achieved': ach / 1e12, 'peak': gemm_peak()[0] / 1e12, 'unit': 'TFLOP/s',
                         'frac': ach / gemm_peak()[0], 'gemm': gemm_peak()[1], 'traffic': _traffic('train88'),
                         'kernel_ms': kms, 'flop_per_launch': flop * n * Pm}}


BLAZE_B = 1024
BLAZE_ID = 'reg1-stoqa9pt-reg2-hrchr82r-selected'


def bench_blazeface(dev, iters, no_cpu):
    """Config 5: the unified BlazeFace + stoqa9pt + hrchr82r graph (reference weights), batch 1024
    frames of 128x128x3 uniform(-1, 1), fp32.  Roofline: the fused ops are each HBM-bound by
    design (depthwise 1.9 FLOP/B), so achieved = the plan's algorithmic bytes (every op's input +
    output map, hpe.blazeface.work_per_image) / the measured time of the whole forward."""
    from hpe import blazeface as BF
    gdir = os.path.join(ROOT, 'tests', 'golden', 'models')
    with open(os.path.join(gdir, BLAZE_ID + '.json')) as fh:
        mc = json.load(fh)['model_config']
    wts = dict(np.load(os.path.join(gdir, BLAZE_ID + '.npz')))
    bf = BF.BlazeFace(mc, wts, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    x = (torch.rand((BLAZE_B, 128, 128, 3), generator=g, device=dev) * 2 - 1).contiguous()
    for _ in range(3):
        bf.forward(x)
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(iters):
        bf.forward(x)
    e1.record()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / iters
    ms = e0.elapsed_time(e1) / iters
    flop, nbytes = BF.work_per_image(bf.plan)
    res = {'workload': 'unified BlazeFace (16 dw/pw blocks, 4 detector heads) + stoqa9pt + hrchr82r '
                       'pose heads, reference weights, batch %d frames 128x128x3 (configs[4])' % BLAZE_B,
           'value': BLAZE_B / wall, 'unit': 'images/sec', 'ms_per_batch': wall * 1e3, 'dtype': 'fp32',
           'data': 'synthetic uniform(-1,1) frames',
           'roofline': {'bound': 'hbm', 'achieved': nbytes * BLAZE_B / (ms * 1e-3) / 1e9,
                        'peak': PEAK_HBM / 1e9, 'unit': 'GB/s',
                        'frac': nbytes * BLAZE_B / (ms * 1e-3) / PEAK_HBM,
                        'traffic': _traffic('blazeface'),
                        'kernel': 'bf_stem_kernel + 16 bf_block_kernel + 2 head GEMMs + 2 regressor '
                                  'programs (hpe_blazeface_forward + hpe_forward)',
                        'kernel_ms': ms, 'bytes_per_launch': nbytes * BLAZE_B,
                        'flop_per_launch': flop * BLAZE_B,
                        'mfma_frac': flop * BLAZE_B / (ms * 1e-3) / PEAK_FP32}}
    if not no_cpu:
        sys.path.insert(0, ROOT)
        from oracle import keras_ref as K
        threads = min(16, os.cpu_count() or 1)
        torch.set_num_threads(threads)
        gr = K.Graph(mc, wts, dtype=torch.float32)
        xs = np.random.default_rng(0).uniform(-1, 1, (8, 128, 128, 3)).astype(np.float32)
        gr.forward(xs)
        t0 = time.perf_counter()
        k = 0
        while time.perf_counter() - t0 < 10.0 or k < 2:
            gr.forward(xs)
            k += 1
        dt = time.perf_counter() - t0
        res['cpu_baseline'] = {'value': k * 8 / dt, 'unit': 'images/sec', 'cores': threads, 'kind': 'port',
                               'sample': '%d forwards x 8 frames (oracle/keras_ref.py torch-CPU fp32), %.1f s'
                                         % (k, dt)}
    return res


def _cpu_name():
    try:
        with open('/proc/cpuinfo') as fh:
            for line in fh:
                if line.startswith('model name'):
                    return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return 'unknown'


def _traffic(kind):
    p = os.path.join(ROOT, 'profiles', 'traffic.json')
    if not os.path.exists(p):
        return None
    try:
        with open(p) as fh:
            return json.load(fh).get(kind, {}).get('hbm_bytes_per_launch')
    except (OSError, ValueError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--no-cpu', action='store_true')
    ap.add_argument('--no-infer', action='store_true')
    ap.add_argument('--no-blaze', action='store_true')
    ap.add_argument('--no-train88', action='store_true')
    a = ap.parse_args()

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group('nccl', device_id=dev)

    import hpe
    from hpe import keras
    hpe.set_seed(42)
    keras.backend.clear_session()
    m = build_train_model(hpe, keras)
    init_w = m.weights_dict()
    eng = m._eng()
    x, y = synth(PER_GPU, 1234 + rank, dev)
    P = H * W
    n_global = PER_GPU * world
    inv_count = 1.0 / (n_global * P * 3)
    stats = torch.zeros((a.steps + a.warmup + 1, 2 + eng.optim_grid()), device=dev)

    def step(i):
        eng.gradient(x, y, P, None, PER_GPU, inv_count, seed=i + 1, img_off=rank * PER_GPU)
        if dist is not None:
            dist.all_reduce(eng.grad)
        eng.optimizer_step(m.optimizer, stats[i])

    for i in range(a.warmup):
        step(i)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    # per-launch timing of the dominant kernel with events on the launch stream (in-loop, cheap)
    starts, ends = [], []
    for i in range(a.steps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        eng.gradient(x, y, P, None, PER_GPU, inv_count, seed=a.warmup + i + 1, img_off=rank * PER_GPU)
        e1.record()
        starts.append(e0)
        ends.append(e1)
        if dist is not None:
            dist.all_reduce(eng.grad)
        eng.optimizer_step(m.optimizer, stats[a.warmup + i])
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    kernel_ms = [s.elapsed_time(e) for s, e in zip(starts, ends)]
    train_ms = float(np.mean(kernel_ms))  # train_step kernel + its reduce kernel
    loss_mse = float(stats[a.warmup + a.steps - 1, 0].item()) / (n_global * P * 3)

    out = None
    if rank == 0:
        ips = n_global * a.steps / dt
        flop_launch = TRAIN_FLOP_POS * PER_GPU * P
        achieved = flop_launch / (train_ms * 1e-3)
        out = {
            'metric': METRIC, 'value': ips, 'unit': 'images/sec', 'n_gpus': world,
            'steps': a.steps, 'warmup': a.warmup, 'ms_per_step': dt * 1e3 / a.steps,
            'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': 'fp32',
            'data': 'synthetic (96x96x96 post-ReLU-like features, random-init weights)',
            'config': {'workload': 'Model-96 create_model(num_filters=360, dropout=0, l2=0.1) '
                                   'training, legacy Adam lr 2.8e-4, 96x96 feature maps '
                                   '(configs[3] per GPU)',
                       'global_batch': n_global, 'positions_per_image': P, 'channels': C,
                       'parallelism': 'dp%d' % world},
            'roofline': {'bound': 'mfma', 'achieved': achieved / 1e12, 'peak': gemm_peak()[0] / 1e12,
                         'unit': 'TFLOP/s', 'frac': achieved / gemm_peak()[0], 'gemm': gemm_peak()[1],
                         'traffic': _traffic('train'),
                         'kernel': {'mlp2': 'mlp2_kernel', 'generic': 'rowprog_kernel'}.get(
                             eng.program('train', P).prog.kind, '?') + ' + reduce_kernel (hpe_train_step + hpe_reduce)',
                         'kernel_ms': train_ms, 'flop_per_launch': flop_launch},
            'train_mse_last_step': loss_mse,
        }
    # ---- inference line (configs[1]) -----------------------------------------------------
    if rank == 0 and not a.no_infer:
        import json as _j
        gdir = os.path.join(ROOT, 'tests', 'golden', 'models')
        with open(os.path.join(gdir, 'hrchr82r.json')) as fh:
            mc = _j.load(fh)['model_config']
        wts = dict(np.load(os.path.join(gdir, 'hrchr82r.npz')))
        im = hpe.model_from_config(mc, wts)
        ie = im._eng()
        xi, _ = synth(INFER_B, 99, dev)
        yo = torch.empty((INFER_B * P, 3), device=dev)
        for _ in range(3):
            ie.forward(xi, P, out=yo)
        torch.cuda.synchronize()
        es = []
        t0 = time.perf_counter()
        n_inf = max(10, a.steps)
        for _ in range(n_inf):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            ie.forward(xi, P, out=yo)
            e1.record()
            es.append((e0, e1))
        torch.cuda.synchronize()
        idt = time.perf_counter() - t0
        ims = float(np.mean([s.elapsed_time(e) for s, e in es]))
        bytes_launch = INFER_BYTES_POS * INFER_B * P
        out['infer'] = {
            'workload': 'Model-96 hrchr82r head (96-32-16-3, reference weights) forward, batch 256, '
                        '96x96 maps (configs[1])',
            'value': INFER_B * n_inf / idt, 'unit': 'images/sec', 'ms_per_batch': idt * 1e3 / n_inf,
            'roofline': {'bound': 'hbm', 'achieved': bytes_launch / (ims * 1e-3) / 1e9,
                         'peak': PEAK_HBM / 1e9, 'unit': 'GB/s',
                         'frac': bytes_launch / (ims * 1e-3) / PEAK_HBM,
                         'traffic': _traffic('infer'),
                         'kernel': {'chain': 'chain_split_kernel (+ guarded chain_fwd_kernel)', 'generic': 'rowprog_kernel'}.get(
                             ie.program('fwd', P).prog.kind, '?') + ' (hpe_forward)',
                         'kernel_ms': ims, 'bytes_per_launch': bytes_launch,
                         'flop_per_launch': INFER_FLOP_POS * INFER_B * P}}
    # ---- Model-88 on 88x88 maps (north_star's second map size) --------------------------------
    if rank == 0 and not a.no_train88:
        out['train88'] = bench_train88(hpe, keras, dev, max(5, min(a.steps, 20)), 2)
    # ---- BlazeFace + both pose heads ----------------------------------
    if rank == 0 and not a.no_blaze:
        out['blazeface'] = bench_blazeface(dev, max(10, a.steps), a.no_cpu or world > 1)
    if rank == 0 and world == 1 and not a.no_cpu:
        cb = cpu_baseline((m.model_config, init_w))
        out['cpu_baseline'] = cb
        out['vs_cpu_baseline'] = out['value'] / cb['value']
    if rank == 0:
        print(json.dumps(out))
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
