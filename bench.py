"""Benchmark: images/sec of the head-pose regressor training step on 96x96 feature maps.

Workload (BASELINE.json configs[3] restated per GPU): the Model-96
``create_model(num_filters=360, dropout 0, l2 0.1)`` graph of Model-96/train_96.py:65-110 with the
legacy Adam optimizer (lr 2.8e-4), synthetic 96x96x96 feature maps (rows of 96 channels, 9216
positions per image, max(0, 0.6 N(0,1) - 0.3)), labels (yaw, pitch, roll) ~ 20 N(0,1) per image,
512 images per GPU per step (weak scaling: global batch 512 x N).  One step = the fused
forward+loss+backward kernel, the workgroup-partial reduce, one RCCL all-reduce of the flat
gradient when N > 1, and the fused Adam kernel — exactly one ``fit`` step of the reference.
Inputs are resident in HBM before the timed region.

Also reported (sub-objects of the one JSON line):
  strong     configs[3] as written: global batch 4096 images split over the N ranks (strong scaling)
  p1         the reference's own regime (train_96.py:134-140,175-183): 1x1 maps (P = 1), batch 128
             and 512, through Model.fit (per-step launches vs the fused epoch kernel), per-step us,
             with the CPU restatement timed at the same batch
  infer      configs[1]: the selected Model-96 head hrchr82r, batch 256 on 96x96 maps, forward only
  train88    Model-88 create_model on 88x88 maps
  blazeface  configs[4]: unified BlazeFace + both pose heads, batch 1024
  blazeface_b1  the reference's own detector call (blazeFaceDetectorH5.py:272, :370): latency of one
             frame (and of 8) per synchronised forward, fused vs per-op plan, CPU oracle beside it
  attn       se_transformer_regr_head (attention_model.py:16-72, checkpoint 12uei1sn: SE + 4-head MHA,
             key_dim 16) on 16x16x88 BlazeFace-tap maps, batch 1024, forward (exact-fp32 MFMA attention
             core, mha_mfma_kernel)
  cpu_baseline  the oracle's torch-CPU fp32 restatement of the headline step on a bounded sample

roofline.frac of every line = its algorithmic work per launch / the dominant kernel's own time
(roofline.dominant_kernel_ms: HIP events the library records around that kernel alone on the launch
stream, averaged over the timed launches; KernelTimer), so it is derivable from the line itself.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
  N > 1 without a torchrun environment: this process starts
  ``python -m torch.distributed.run --nproc-per-node N ... bench.py`` as a CHILD (before anything
  touches the GPU) and exits with its code; under torchrun (RANK / WORLD_SIZE set) it is one rank.
"""
import argparse
import json
import math
import os
import socket
import subprocess
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
STRONG_GLOBAL = 4096
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


# ---------------------------------------------------------------------------------------------
# N-rank launch (no GPU call before this decision)
# ---------------------------------------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_plan(gpus, argv, env):
    """Command line of the N-rank child launch, or None when this process is itself the job
    (N == 1, or already a torchrun rank).  Pure: touches no device."""
    if gpus <= 1 or 'WORLD_SIZE' in env:
        return None
    return [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', str(gpus),
            '--master-addr', '127.0.0.1', '--master-port', str(_free_port()),
            os.path.abspath(__file__)] + list(argv)


KFD_NODES = '/sys/class/kfd/kfd/topology/nodes'


def visible_gpus(env=None, kfd=KFD_NODES):
    """GPUs this job may use, counted WITHOUT the HIP runtime (the launcher must not initialise a
    device before its ranks start): the visible-devices list when one is set
    (ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES, the most restrictive wins),
    else the KFD topology nodes that are GPUs (simd_count > 0).  0 when neither is available."""
    env = os.environ if env is None else env
    lists = [env[k] for k in ('ROCR_VISIBLE_DEVICES', 'HIP_VISIBLE_DEVICES', 'CUDA_VISIBLE_DEVICES')
             if env.get(k) is not None]
    n_kfd = 0
    try:
        for node in os.listdir(kfd):
            try:
                with open(os.path.join(kfd, node, 'properties')) as fh:
                    props = dict(l.split()[:2] for l in fh if len(l.split()) >= 2)
            except OSError:
                continue
            if int(props.get('simd_count', '0')) > 0:
                n_kfd += 1
    except OSError:
        pass
    counts = [len([d for d in l.split(',') if d.strip() != '']) for l in lists]
    if counts:
        return min(counts + ([n_kfd] if n_kfd else []))
    return n_kfd


def spawn_ranks(gpus, argv):
    """Run ``gpus`` ranks as a child torchrun job; returns its exit code.  The GPUs are counted
    from the visible-devices env / KFD sysfs (visible_gpus), never through HIP: this process only
    launches the ranks."""
    n_dev = visible_gpus()
    if n_dev < gpus:
        print('bench.py: --gpus %d requested but only %d GPU(s) visible' % (gpus, n_dev), file=sys.stderr)
        return 2
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    return subprocess.call(launch_plan(gpus, argv, {}), env=env)


# ---------------------------------------------------------------------------------------------
# workloads
# ---------------------------------------------------------------------------------------------
def build_train_model(keras, F_=F, l2=0.1, dropout=0.0):
    """create_model() of Model-96/train_96.py:65-110 with num_filters=F_, dropout, l2."""
    reg = keras.regularizers.l2(l2)
    inp = keras.Input(shape=(None, None, 96))
    x1 = keras.layers.Conv2D(filters=F_, kernel_size=1, padding='same', activation='tanh',
                             kernel_initializer=keras.initializers.GlorotUniform(),
                             bias_regularizer=reg, kernel_regularizer=reg)(inp)
    x1 = keras.layers.SpatialDropout2D(dropout)(x1)
    out = keras.layers.Conv2D(filters=3, kernel_size=1, padding='same', activation=None,
                              kernel_initializer=keras.initializers.GlorotUniform(),
                              bias_regularizer=reg, kernel_regularizer=reg)(x1)
    out = keras.layers.SpatialDropout2D(dropout)(out)
    m = keras.Model(inputs=inp, outputs=out)
    m.compile(optimizer=keras.optimizers.Adam(learning_rate=0.00028), loss='mse', metrics=['mae'])
    return m


def build_complex_88(keras):
    """create_model_complex(1e-6, 1e-4) of Model-88/attention_model.py:97-169 (the drop-in builder
    in head-pose-estimation-model_amd/Model-88/attention_model.py), compiled as train_88.py:323-328
    (legacy SGD lr 2.8e-4, mse, mae)."""
    import importlib.util
    path = os.path.join(ROOT, 'head-pose-estimation-model_amd', 'Model-88', 'attention_model.py')
    spec = importlib.util.spec_from_file_location('hpe_attention_model_88', path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    keras.backend.clear_session()
    m = mod.create_model_complex(1e-6, 1e-4)
    m.compile(optimizer=keras.optimizers.SGD(learning_rate=0.00028), loss='mse', metrics=['mae'])
    return m


def synth(n_img, seed, device, P=H * W, c=C):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    x = torch.randn((n_img * P, c), generator=g, device=device, dtype=torch.float32)
    x = torch.clamp_min(0.6 * x - 0.3, 0.0)
    y = 20.0 * torch.randn((n_img, 3), generator=g, device=device, dtype=torch.float32)
    return x.contiguous(), y.contiguous()


class KernelTimer:
    """HIP events around each launch's dominant kernel only (libhpe.so hpe_kernel_timing: recorded
    by the library on the launch stream around the fp16-split kernel, not its early-exit exact twin
    nor the reduce)."""

    def __init__(self, n):
        from hpe import _lib
        self.lib, self.n = _lib.load(), n

    def __enter__(self):
        from hpe import _lib
        _lib.check(self.lib.hpe_kernel_timing(self.n), 'hpe_kernel_timing')
        return self

    def __exit__(self, *exc):
        import ctypes
        buf = (ctypes.c_float * self.n)()
        k = self.lib.hpe_kernel_times(buf, self.n)
        self.lib.hpe_kernel_timing(0)
        self.ms = [float(v) for v in buf[:max(k, 0)]]
        return False

    def mean(self):
        return float(np.mean(self.ms)) if self.ms else float('nan')


def run_train(eng, opt, x, y, P, n_local, n_global, rank, world, steps, warmup, dist):
    """Timed training steps (barrier + synchronize on both sides, max over ranks).  Returns
    (seconds, mean ms of the train_step + reduce launches measured with HIP events on the launch
    stream, mse of the last step, mean ms of the dominant kernel alone (KernelTimer))."""
    inv_count = 1.0 / (n_global * P * 3)
    stats = torch.zeros((steps + warmup + 1, 2 + eng.optim_grid()), device=x.device)
    for i in range(warmup):
        eng.gradient(x, y, P, None, n_local, inv_count, seed=i + 1, img_off=rank * n_local)
        if dist is not None:
            dist.all_reduce(eng.grad)
        eng.optimizer_step(opt, stats[i])
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    kt = KernelTimer(steps)
    t0 = time.perf_counter()
    marks = []
    with kt:
        for i in range(steps):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            eng.gradient(x, y, P, None, n_local, inv_count, seed=warmup + i + 1, img_off=rank * n_local)
            e1.record()
            marks.append((e0, e1))
            if dist is not None:
                dist.all_reduce(eng.grad)
            eng.optimizer_step(opt, stats[warmup + i])
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], device=x.device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    kms = float(np.mean([a.elapsed_time(b) for a, b in marks]))
    mse = float(stats[warmup + steps - 1, 0].item()) / (n_global * P * 3)
    return dt, kms, mse, kt.mean()


def train_kernel_name(eng, P, rows=0):
    """The kernel libhpe.so runs for a training launch of this program over `rows` rows
    (csrc/hpe_mlp2.hip launch_pair / pick_r: the row-parallel mlp2r_kernel for F <= 64 on launches of
    >= 2^15 rows, else mlp2_kernel; the fp16-split instantiations unless exact fp32 is forced)."""
    from hpe.compiler import ACTS
    prog = eng.program('train', P).prog
    if prog.kind == 'res':
        return 'res_train_kernel'
    if prog.kind != 'mlp2':
        return 'rowprog_kernel'
    if os.environ.get('HPE_EXACT_FP32') == '1':
        return 'mlp2_kernel (exact fp32)'
    i = prog.info
    if (os.environ.get('HPE_MLP2_ROWS') != '0' and rows >= 1 << 15 and i['F'] <= 64 and i['act2'] == 0 and
            i['act'] in (ACTS['tanh'], ACTS['softsign']) and (i['cin'] == 88 or (i['cin'] + 7) // 8 * 4 == 48)):
        return 'mlp2r_kernel'
    return 'mlp2_kernel'


def _threads_for_cpu(probe):
    """Thread count for the CPU restatement: every CPU this process may run on
    (os.sched_getaffinity), unless the box's OMP_NUM_THREADS share runs the probe faster (an
    oversubscribed cgroup quota).  Returns (threads, {threads: probe seconds})."""
    try:
        allowed = len(os.sched_getaffinity(0))
    except AttributeError:
        allowed = os.cpu_count() or 1
    cands = sorted({allowed, int(os.environ.get('OMP_NUM_THREADS', allowed) or allowed)})
    times = {}
    for t in cands:
        torch.set_num_threads(t)
        probe()
        t0 = time.perf_counter()
        probe()
        times[t] = time.perf_counter() - t0
    best = min(times, key=times.get)
    torch.set_num_threads(best)
    return best, times


def cpu_baseline(weights_cfg, steps_budget_s=12.0):
    """Oracle (torch-CPU fp32 restatement of Keras semantics) timed on a bounded sample:
    training steps on 2 images of 96x96 (18,432 rows) each, legacy Adam, as many as fit in
    ~steps_budget_s."""
    sys.path.insert(0, ROOT)
    from oracle import keras_ref as K
    mc, w = weights_cfg
    g = K.Graph(mc, w, dtype=torch.float32)
    opt = K.LegacyOptimizer('adam', 2.8e-4)
    rng = np.random.default_rng(0)
    n = 2
    x = np.maximum(0.0, 0.6 * rng.standard_normal((n, H, W, C)) - 0.3).astype(np.float32)
    y = (20 * rng.standard_normal((n, 3))).astype(np.float32)
    xt, yt = torch.from_numpy(x), torch.from_numpy(y)
    threads, probes = _threads_for_cpu(lambda: K.train_step(g, opt, xt, yt))
    t0 = time.perf_counter()
    steps = 0
    while time.perf_counter() - t0 < steps_budget_s or steps < 2:
        K.train_step(g, opt, xt, yt)
        steps += 1
    dt = time.perf_counter() - t0
    return {'value': steps * n / dt, 'unit': 'images/sec', 'cores': threads, 'kind': 'port',
            'sample': '%d training steps x %d images of 96x96x96 (create_model(360), Adam, '
                      'torch-CPU fp32 restatement, oracle/keras_ref.py), %.1f s' % (steps, n, dt),
            'cpu': _cpu_name(), 'os_cpu_count': os.cpu_count(),
            'thread_probe_s': {str(k): round(v, 4) for k, v in probes.items()}}


class _EpochTimer:
    """keras-style callback: wall time of every epoch of fit (per-epoch host work included)."""

    def __init__(self):
        self.model = None
        self.params = {}
        self.times = []

    def set_model(self, m):
        self.model = m

    def set_params(self, p):
        self.params = p

    def on_train_begin(self, logs=None):
        pass

    def on_train_end(self, logs=None):
        pass

    def on_epoch_begin(self, epoch, logs=None):
        self.t0 = time.perf_counter()

    def on_epoch_end(self, epoch, logs=None):
        self.times.append(time.perf_counter() - self.t0)


def bench_p1(keras, batches=(128, 512), n_rows=1 << 20, epochs=3, no_cpu=False):
    """The reference's training regime (train_96.py:134-140,175-183): create_model(360), Adam,
    1x1 feature maps (P = 1), 80/20 split with validation each epoch, batch 128 (the reference's)
    and 512, through Model.fit.  Per-step time = median epoch wall time / steps per epoch, for the
    per-step launch path (train_step + reduce + optimizer launches per step, HPE_FIT_FUSED=0) and
    the fused epoch kernel (one launch per epoch; default)."""
    import hpe
    from hpe.data import train_test_split
    rng = np.random.default_rng(0)
    x = np.maximum(0.0, 0.6 * rng.standard_normal((n_rows, 1, 1, C)) - 0.3).astype(np.float32)
    y = (20 * rng.standard_normal((n_rows, 1, 1, 3))).astype(np.float32)
    tx, vx, ty, vy = train_test_split(x, y, test_size=0.2, random_state=42)
    out = {'workload': 'Model-96 create_model(360, dropout 0, l2 0.1), legacy Adam, synthetic 1x1x96 '
                       'features, %d rows (80/20 split, validation every epoch), Model.fit' % n_rows,
           'unit': 'us/step', 'lines': {}}
    prev = os.environ.get('HPE_FIT_FUSED')
    try:
        for bs in batches:
            steps = math.ceil(tx.shape[0] / bs)
            # the fused epoch splits a step over hidden units only (<= 12 workgroups at F = 360):
            # above batch 256 fit runs the per-step launches (FIT_FUSED_AUTO_MAX), so only those
            # are measured there
            for mode in ('per_step', 'fused_epoch') if bs <= 256 else ('per_step',):
                os.environ['HPE_FIT_FUSED'] = '0' if mode == 'per_step' else '1'
                hpe.set_seed(42)
                keras.backend.clear_session()
                m = build_train_model(keras)
                tm = _EpochTimer()
                ep = 1 if mode == 'per_step' and bs <= 128 else epochs
                m.fit(tx, ty, batch_size=bs, epochs=ep + 1, validation_data=(vx, vy), callbacks=[tm],
                      verbose=0)
                t_ep = float(np.median(tm.times[1:]))
                out['lines']['%s_b%d' % (mode, bs)] = {
                    'us_per_step': t_ep / steps * 1e6, 'images_per_sec': tx.shape[0] / t_ep,
                    'epoch_s': t_ep, 'steps_per_epoch': steps, 'epochs_timed': len(tm.times) - 1,
                    'fused': bool(getattr(m, '_last_fit_fused', False)),
                    'final_loss': float(m.history.history['loss'][-1])}
            if bs <= 256:
                ps, fe = out['lines']['per_step_b%d' % bs], out['lines']['fused_epoch_b%d' % bs]
                out['lines']['speedup_b%d' % bs] = ps['us_per_step'] / fe['us_per_step']
    finally:
        if prev is None:
            os.environ.pop('HPE_FIT_FUSED', None)
        else:
            os.environ['HPE_FIT_FUSED'] = prev
    # Model-88 in the reference's own regime on the reference's own training data (train_88.py:
    # 20-62, 270): create_model 88-64 softsign, dropout 1e-4, l2 1e-6, legacy SGD lr 2.8e-4, batch 128
    d88 = np.load(os.path.join(ROOT, 'tests', 'golden', 'data', 'BIWI_Train_Enlarged_features_88_0.7_1.npz'))
    x88 = d88['features'].reshape(-1, 1, 1, 88).astype(np.float32)
    y88 = d88['poses'].reshape(-1, 1, 1, 3).astype(np.float32)
    t88x, v88x, t88y, v88y = train_test_split(x88, y88, test_size=0.2, random_state=42)
    try:
        for mode in ('per_step', 'fused_epoch'):
            os.environ['HPE_FIT_FUSED'] = '0' if mode == 'per_step' else '1'
            hpe.set_seed(42)
            keras.backend.clear_session()
            reg = keras.regularizers.l2(1e-6)
            inp = keras.Input(shape=(None, None, 88))
            h = keras.layers.Conv2D(64, 1, activation='softsign', kernel_regularizer=reg)(inp)
            h = keras.layers.SpatialDropout2D(1e-4)(h)
            o = keras.layers.Conv2D(3, 1, kernel_regularizer=reg)(h)
            o = keras.layers.SpatialDropout2D(1e-4)(o)
            m = keras.Model(inp, o)
            m.compile(optimizer=keras.optimizers.SGD(learning_rate=0.00028), loss='mse', metrics=['mae'])
            tm = _EpochTimer()
            m.fit(t88x, t88y, batch_size=128, epochs=21, validation_data=(v88x, v88y), callbacks=[tm], verbose=0)
            steps = math.ceil(t88x.shape[0] / 128)
            t_ep = float(np.median(tm.times[1:]))
            out['lines']['model88_real_%s_b128' % mode] = {
                'data': 'BIWI_Train_Enlarged_features_88 (10,284 rows, 8,227 train / 2,057 validation)',
                'us_per_step': t_ep / steps * 1e6, 'images_per_sec': t88x.shape[0] / t_ep, 'epoch_s': t_ep,
                'steps_per_epoch': steps, 'epochs_timed': len(tm.times) - 1,
                'fused': bool(getattr(m, '_last_fit_fused', False))}
    finally:
        if prev is None:
            os.environ.pop('HPE_FIT_FUSED', None)
        else:
            os.environ['HPE_FIT_FUSED'] = prev
    # configs[2]: Model-88 create_model, legacy Adam, batch 512 (BASELINE.json), same data; fit runs
    # it through the per-step launches (batch > FIT_FUSED_AUTO_MAX), the only mode measured
    try:
        for mode in ('per_step',):
            os.environ['HPE_FIT_FUSED'] = '0' if mode == 'per_step' else '1'
            hpe.set_seed(42)
            keras.backend.clear_session()
            reg = keras.regularizers.l2(1e-6)
            inp = keras.Input(shape=(None, None, 88))
            h = keras.layers.Conv2D(64, 1, activation='softsign', kernel_regularizer=reg)(inp)
            h = keras.layers.SpatialDropout2D(1e-4)(h)
            o = keras.layers.Conv2D(3, 1, kernel_regularizer=reg)(h)
            o = keras.layers.SpatialDropout2D(1e-4)(o)
            m = keras.Model(inp, o)
            m.compile(optimizer=keras.optimizers.Adam(learning_rate=0.00028), loss='mse', metrics=['mae'])
            tm = _EpochTimer()
            m.fit(t88x, t88y, batch_size=512, epochs=21, validation_data=(v88x, v88y), callbacks=[tm], verbose=0)
            steps = math.ceil(t88x.shape[0] / 512)
            t_ep = float(np.median(tm.times[1:]))
            out['lines']['model88_adam_%s_b512' % mode] = {
                'data': 'BIWI_Train_Enlarged_features_88, configs[2]: Adam, batch 512',
                'us_per_step': t_ep / steps * 1e6, 'images_per_sec': t88x.shape[0] / t_ep, 'epoch_s': t_ep,
                'steps_per_epoch': steps, 'epochs_timed': len(tm.times) - 1,
                'fused': bool(getattr(m, '_last_fit_fused', False))}
    finally:
        if prev is None:
            os.environ.pop('HPE_FIT_FUSED', None)
        else:
            os.environ['HPE_FIT_FUSED'] = prev
    # train_88.py's own default graph: create_model_complex(1e-6, 1e-4) (attention_model.py:97-169,
    # train_88.py:309), legacy SGD 2.8e-4, batch 128, on the same data: the generic row program
    hpe.set_seed(42)
    cmc = build_complex_88(keras)
    tm = _EpochTimer()
    cmc.fit(t88x, t88y, batch_size=128, epochs=6, validation_data=(v88x, v88y), callbacks=[tm], verbose=0)
    steps = math.ceil(t88x.shape[0] / 128)
    t_ep = float(np.median(tm.times[1:]))
    out['lines']['model88_complex_b128'] = {
        'data': 'BIWI_Train_Enlarged_features_88 (train_88.py:270), create_model_complex(1e-6, 1e-4), SGD 2.8e-4',
        'us_per_step': t_ep / steps * 1e6, 'images_per_sec': t88x.shape[0] / t_ep, 'epoch_s': t_ep,
        'steps_per_epoch': steps, 'epochs_timed': len(tm.times) - 1,
        'fused': bool(getattr(cmc, '_last_fit_fused', False)),
        'kernel': cmc._eng().program('train', 1).prog.kind + ' row program'}
    if not no_cpu:
        sys.path.insert(0, ROOT)
        from oracle import keras_ref as K
        keras.backend.clear_session()
        cmc = build_complex_88(keras)
        g = K.Graph(cmc.model_config, cmc.weights_dict(), dtype=torch.float32)
        opt = K.LegacyOptimizer('sgd', 2.8e-4)
        xb, yb = torch.from_numpy(t88x[:128]), torch.from_numpy(t88y[:128].reshape(128, 3))
        threads, _ = _threads_for_cpu(lambda: K.train_step(g, opt, xb, yb))
        t0 = time.perf_counter()
        k = 0
        while time.perf_counter() - t0 < 4.0 or k < 5:
            K.train_step(g, opt, xb, yb)
            k += 1
        dt = (time.perf_counter() - t0) / k
        out['lines']['model88_complex_b128']['cpu_baseline'] = {
            'us_per_step': dt * 1e6, 'cores': threads, 'kind': 'port',
            'sample': '%d SGD steps of batch 128 (oracle/keras_ref.py torch-CPU fp32)' % k}
    if not no_cpu:
        sys.path.insert(0, ROOT)
        from oracle import keras_ref as K
        keras.backend.clear_session()
        m = build_train_model(keras)
        g = K.Graph(m.model_config, m.weights_dict(), dtype=torch.float32)
        opt = K.LegacyOptimizer('adam', 2.8e-4)
        res = {}
        for bs in batches:
            xb, yb = torch.from_numpy(tx[:bs]), torch.from_numpy(ty[:bs].reshape(bs, 3))
            threads, _ = _threads_for_cpu(lambda: K.train_step(g, opt, xb, yb))
            t0 = time.perf_counter()
            k = 0
            while time.perf_counter() - t0 < 4.0 or k < 5:
                K.train_step(g, opt, xb, yb)
                k += 1
            dt = (time.perf_counter() - t0) / k
            res['b%d' % bs] = {'us_per_step': dt * 1e6, 'images_per_sec': bs / dt, 'cores': threads,
                               'kind': 'port', 'sample': '%d steps of batch %d (oracle/keras_ref.py '
                                                         'torch-CPU fp32)' % (k, bs)}
        out['cpu_baseline'] = res
    return out


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
    x, y = synth(n, 88, dev, P=Pm, c=88)
    dt, kms, _, dom_ms = run_train(eng, m.optimizer, x, y, Pm, n, n, 0, 1, steps, warmup, None)
    flop = 2 * (88 * 64 + 64 * 3) * 2 + 2 * 64 * 3            # fwd + dW + dX(layer 2) per position
    ach = flop * n * Pm / (dom_ms * 1e-3)
    return {'workload': 'Model-88 create_model (88-64 softsign-3, dropout 1e-4, l2 1e-6) training, legacy Adam, '
                        '512 images of 88x88 feature maps',
            'value': n * steps / dt, 'unit': 'images/sec', 'ms_per_step': dt * 1e3 / steps, 'dtype': 'fp32',
            'kernel': train_kernel_name(eng, Pm, n * Pm),
            'roofline': {'bound': 'mfma', 'achieved': ach / 1e12, 'peak': gemm_peak()[0] / 1e12, 'unit': 'TFLOP/s',
                         'frac': ach / gemm_peak()[0], 'gemm': gemm_peak()[1], 'traffic': _traffic('train88'),
                         'dominant_kernel_ms': dom_ms, 'step_kernels_ms': kms, 'flop_per_launch': flop * n * Pm}}


BLAZE_B = 1024
BLAZE_ID = 'reg1-stoqa9pt-reg2-hrchr82r-selected'


def bench_blazeface(dev, iters, no_cpu):
    """Config 5: the unified BlazeFace + stoqa9pt + hrchr82r graph (reference weights), batch 1024
    frames of 128x128x3 uniform(-1, 1), fp32.  Roofline: achieved = the frame's compulsory HBM
    bytes (hpe.blazeface.compulsory_bytes_per_image: input, detector outputs, taps, pose maps) /
    the measured time of the whole forward; plan_bytes (every launch's input + output maps,
    hpe.blazeface.work_per_image) and mfma_frac alongside."""
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
    flop, plan_bytes = BF.work_per_image(bf.plan)
    nbytes = BF.compulsory_bytes_per_image(bf.plan)
    res = {'workload': 'unified BlazeFace (16 dw/pw blocks, 4 detector heads) + stoqa9pt + hrchr82r '
                       'pose heads, reference weights, batch %d frames 128x128x3 (configs[4])' % BLAZE_B,
           'value': BLAZE_B / wall, 'unit': 'images/sec', 'ms_per_batch': wall * 1e3, 'dtype': 'fp32',
           'data': 'synthetic uniform(-1,1) frames',
           # 173 FLOP per compulsory byte: compute-bound.  frac on the FLOPs against the ceiling the
           # pointwise convs run on (fp32 products as 3 fp16 MFMA products: dense fp16 / 3); the HBM
           # fraction on COMPULSORY bytes (input frame + detector outputs + taps + pose maps, once
           # each) and on plan_bytes (the launches' input / output maps) beside it
           'roofline': {'bound': 'mfma', 'achieved': flop * BLAZE_B / (ms * 1e-3) / 1e12,
                        'peak': PEAK_F16 / 3 / 1e12, 'unit': 'TFLOP/s',
                        'frac': flop * BLAZE_B / (ms * 1e-3) / (PEAK_F16 / 3),
                        'peak_basis': 'fp32 products as 3 fp16 MFMA products: 2.5 PFLOP/s dense fp16 / 3 '
                                      '(depthwise FMAs, a sixth of the FLOPs, run on VALU)',
                        'traffic': _traffic('blazeface'),
                        'hbm_frac': nbytes * BLAZE_B / (ms * 1e-3) / PEAK_HBM,
                        'hbm_achieved_GBps': nbytes * BLAZE_B / (ms * 1e-3) / 1e9,
                        'kernel': 'bf_front_kernel (stem + 64x64 / 32x32 blocks) + bf_stage_kernel (16x16 / 8x8 '
                                  'blocks + detector heads) + 2 pose regressor programs (hpe_blazeface_forward '
                                  '+ hpe_forward), whole forward',
                        'kernel_ms': ms, 'bytes_per_launch': nbytes * BLAZE_B,
                        'plan_bytes': plan_bytes * BLAZE_B,
                        'plan_frac': plan_bytes * BLAZE_B / (ms * 1e-3) / PEAK_HBM,
                        'flop_per_launch': flop * BLAZE_B}}
    if not no_cpu:
        sys.path.insert(0, ROOT)
        from oracle import keras_ref as K
        gr = K.Graph(mc, wts, dtype=torch.float32)
        xs = np.random.default_rng(0).uniform(-1, 1, (8, 128, 128, 3)).astype(np.float32)
        threads, _ = _threads_for_cpu(lambda: gr.forward(xs))
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


def bench_blazeface_b1(dev, no_cpu, batches=(1, 8), reps=50):
    """The reference's own detector call (BlazePoser/blazeFaceDetectorH5.py:272, one frame per call
    in the webcam loop :370): frames -> detector outputs + poses latency at batch 1 and 8, median of
    `reps` synchronised forwards, for the default plan (bf_front_kernel + bf_stage_kernel + the two
    pose programs) and the per-op plan (one launch per layer), beside the oracle's CPU latency."""
    from hpe import blazeface as BF
    gdir = os.path.join(ROOT, 'tests', 'golden', 'models')
    with open(os.path.join(gdir, BLAZE_ID + '.json')) as fh:
        mc = json.load(fh)['model_config']
    wts = dict(np.load(os.path.join(gdir, BLAZE_ID + '.npz')))
    plans = {'fused': BF.BlazeFace(mc, wts, device=dev),
             'per_op': BF.BlazeFace(mc, wts, device=dev, stage=False, front=False)}
    res = {'workload': 'unified BlazeFace + stoqa9pt + hrchr82r pose heads, reference weights, one '
                       'synchronised forward per call (frames -> detector outputs + pose maps)',
           'unit': 'ms per call (median of %d)' % reps, 'lines': {}}
    g = torch.Generator(device=dev)
    g.manual_seed(6)
    for n in batches:
        x = (torch.rand((n, 128, 128, 3), generator=g, device=dev) * 2 - 1).contiguous()
        for name, bf in plans.items():
            for _ in range(5):
                bf.forward(x)
            torch.cuda.synchronize()
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                bf.forward(x)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            ms = 1e3 * float(np.median(ts))
            res['lines']['%s_b%d' % (name, n)] = {'ms': ms, 'frames_per_sec': n / ms * 1e3}
    res['value_ms_b1'] = min(res['lines']['fused_b1']['ms'], res['lines']['per_op_b1']['ms'])
    res['plan_b1'] = 'fused' if res['lines']['fused_b1']['ms'] <= res['lines']['per_op_b1']['ms'] else 'per_op'
    if not no_cpu:
        sys.path.insert(0, ROOT)
        from oracle import keras_ref as K
        gr = K.Graph(mc, wts, dtype=torch.float32)
        xs = np.random.default_rng(1).uniform(-1, 1, (1, 128, 128, 3)).astype(np.float32)
        threads, _ = _threads_for_cpu(lambda: gr.forward(xs))
        ts = []
        t_end = time.perf_counter() + 5.0
        while time.perf_counter() < t_end or len(ts) < 3:
            t0 = time.perf_counter()
            gr.forward(xs)
            ts.append(time.perf_counter() - t0)
        res['cpu_baseline'] = {'value': 1e3 * float(np.median(ts)), 'unit': 'ms per frame (batch 1)',
                               'cores': threads, 'kind': 'port',
                               'sample': '%d batch-1 forwards (oracle/keras_ref.py torch-CPU fp32), median'
                                         % len(ts)}
    return res


ATTN_B = 1024
ATTN_ID = '12uei1sn'


def bench_attn(dev, iters):
    """se_transformer_regr_head (Model-88/attention_model.py:16-72) on H x W = 16 x 16 maps of 88
    channels (a BlazeFace re_lu_10 tap per frame), checkpoint 12uei1sn (SE r=8, MultiHeadAttention 4
    heads x key_dim 16, LayerNorms, feed-forward, 1x1-conv head), batch 1024 images: hpe_se_gate ->
    program B (q|k|v) -> hpe_mha -> program D.  Roofline of the attention core (the dominant FLOPs:
    4 P^2 D per head per image, exact fp32 MFMA) against the dense fp32 MFMA peak; the row
    programs and the SE gate are HBM-bound (algorithmic bytes: every stage's input + output rows)."""
    from hpe.spatial import SpatialHead
    gdir = os.path.join(ROOT, 'tests', 'golden', 'models')
    with open(os.path.join(gdir, ATTN_ID + '.json')) as fh:
        mc = json.load(fh)['model_config']
    wts = dict(np.load(os.path.join(gdir, ATTN_ID + '.npz')))
    sh = SpatialHead(mc, wts, dev)
    P, Cc = 16 * 16, sh.C
    H, D = sh.plan.mha['H'], sh.plan.mha['D']
    x, _ = synth(ATTN_B, 77, dev, P=P, c=Cc)
    for _ in range(3):
        y = sh.forward(x, P)
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(iters):
        y = sh.forward(x, P)
    e1.record()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / iters
    ms = e0.elapsed_time(e1) / iters
    attn_flop = 4.0 * P * P * D * H * ATTN_B
    qkv_w = sh.qkv.program('fwd', P).prog.C_out
    rows = ATTN_B * P
    nbytes = 4 * rows * (Cc * 3 + qkv_w + (Cc + 3 * H * D) + (Cc + H * D) + y.shape[1])
    return {'workload': 'se_transformer_regr_head (checkpoint %s: SE + MHA %d heads x key_dim %d) forward on '
                        '16x16x%d maps, batch %d images (attention_model.py:16-72)' % (ATTN_ID, H, D, Cc, ATTN_B),
            'value': ATTN_B / wall, 'unit': 'images/sec', 'ms_per_batch': wall * 1e3, 'dtype': 'fp32',
            'roofline': {'bound': 'mfma', 'achieved': attn_flop / (ms * 1e-3) / 1e12, 'peak': PEAK_FP32 / 1e12,
                         'unit': 'TFLOP/s', 'frac': attn_flop / (ms * 1e-3) / PEAK_FP32,
                         'kernel': 'se_gate_kernel + rowprog (q|k|v) + mha_mfma_kernel<16> (exact fp32 MFMA) + '
                                   'rowprog (head), whole forward; peak = dense fp32 MFMA',
                         'kernel_ms': ms, 'attn_flop_per_launch': attn_flop,
                         'hbm_bytes_algorithmic': nbytes, 'hbm_frac': nbytes / (ms * 1e-3) / PEAK_HBM}}


def bench_infer(hpe, dev, steps):
    """configs[1]: hrchr82r forward, batch 256 of 96x96 maps."""
    gdir = os.path.join(ROOT, 'tests', 'golden', 'models')
    with open(os.path.join(gdir, 'hrchr82r.json')) as fh:
        mc = json.load(fh)['model_config']
    wts = dict(np.load(os.path.join(gdir, 'hrchr82r.npz')))
    im = hpe.model_from_config(mc, wts)
    ie = im._eng()
    P = H * W
    xi, _ = synth(INFER_B, 99, dev)
    yo = torch.empty((INFER_B * P, 3), device=dev)
    for _ in range(3):
        ie.forward(xi, P, out=yo)
    torch.cuda.synchronize()
    es = []
    n_inf = max(10, steps)
    kt = KernelTimer(n_inf)
    t0 = time.perf_counter()
    with kt:
        for _ in range(n_inf):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            ie.forward(xi, P, out=yo)
            e1.record()
            es.append((e0, e1))
        torch.cuda.synchronize()
    idt = time.perf_counter() - t0
    fwd_ms = float(np.mean([s.elapsed_time(e) for s, e in es]))
    ims = kt.mean()
    bytes_launch = INFER_BYTES_POS * INFER_B * P
    return {
        'workload': 'Model-96 hrchr82r head (96-32-16-3, reference weights) forward, batch 256, '
                    '96x96 maps (configs[1])',
        'value': INFER_B * n_inf / idt, 'unit': 'images/sec', 'ms_per_batch': idt * 1e3 / n_inf,
        'roofline': {'bound': 'hbm', 'achieved': bytes_launch / (ims * 1e-3) / 1e9,
                     'peak': PEAK_HBM / 1e9, 'unit': 'GB/s',
                     'frac': bytes_launch / (ims * 1e-3) / PEAK_HBM,
                     'traffic': _traffic('infer'),
                     'kernel': {'chain': 'chain_split_kernel (+ guarded chain_fwd_kernel)',
                                'generic': 'rowprog_kernel'}.get(ie.program('fwd', P).prog.kind, '?')
                     + ' (hpe_forward)',
                     'dominant_kernel_ms': ims, 'forward_ms': fwd_ms, 'bytes_per_launch': bytes_launch,
                     'flop_per_launch': INFER_FLOP_POS * INFER_B * P}}


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


def parse(argv):
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--no-cpu', action='store_true')
    ap.add_argument('--no-infer', action='store_true')
    ap.add_argument('--no-blaze', action='store_true')
    ap.add_argument('--no-train88', action='store_true')
    ap.add_argument('--no-strong', action='store_true')
    ap.add_argument('--no-p1', action='store_true')
    ap.add_argument('--no-attn', action='store_true')
    ap.add_argument('--only', default='', help='comma list of lines to run (train,strong,p1,infer,train88,blazeface,blazeface_b1,attn)')
    return ap.parse_args(argv)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    if launch_plan(a.gpus, argv, os.environ) is not None:
        sys.exit(spawn_ranks(a.gpus, argv))
    only = set(x for x in a.only.split(',') if x)

    def want(name, flag=False):
        return (name in only) if only else not flag

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world != a.gpus and 'WORLD_SIZE' in os.environ:
        print('bench.py: --gpus %d but WORLD_SIZE=%d; using WORLD_SIZE' % (a.gpus, world), file=sys.stderr)
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
    m = build_train_model(keras)
    init_w = m.weights_dict()
    eng = m._eng()
    P = H * W
    n_global = PER_GPU * world
    out = {'metric': METRIC, 'unit': 'images/sec', 'n_gpus': world, 'steps': a.steps, 'warmup': a.warmup,
           'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': 'fp32',
           'data': 'synthetic (96x96x96 post-ReLU-like features, random-init weights)',
           'config': {'workload': 'Model-96 create_model(num_filters=360, dropout=0, l2=0.1) '
                                  'training, legacy Adam lr 2.8e-4, 96x96 feature maps '
                                  '(configs[3] per GPU: 512 images per rank)',
                      'global_batch': n_global, 'per_gpu_batch': PER_GPU, 'positions_per_image': P,
                      'channels': C, 'parallelism': 'dp%d' % world},
           'world_size_seen': dist.get_world_size() if dist is not None else 1,
           'backend': dist.get_backend() if dist is not None else 'none (single process)'}
    if want('train'):
        x, y = synth(PER_GPU, 1234 + rank, dev)
        dt, train_ms, mse, dom_ms = run_train(eng, m.optimizer, x, y, P, PER_GPU, n_global, rank, world,
                                              a.steps, a.warmup, dist)
        del x, y
        flop_launch = TRAIN_FLOP_POS * PER_GPU * P
        achieved = flop_launch / (dom_ms * 1e-3)
        out.update({
            'value': n_global * a.steps / dt, 'ms_per_step': dt * 1e3 / a.steps,
            'roofline': {'bound': 'mfma', 'achieved': achieved / 1e12, 'peak': gemm_peak()[0] / 1e12,
                         'unit': 'TFLOP/s', 'frac': achieved / gemm_peak()[0], 'gemm': gemm_peak()[1],
                         'traffic': _traffic('train'),
                         'kernel': train_kernel_name(eng, P, PER_GPU * P),
                         'dominant_kernel_ms': dom_ms,
                         'frac_from': 'flop_per_launch / dominant_kernel_ms (HIP events around the dominant '
                                      'kernel alone, every timed step, on the launch stream) / peak',
                         'step_kernels_ms': train_ms,
                         'step_kernels': 'hpe_train_step (dominant kernel + exact twin early exit) + hpe_reduce',
                         'flop_per_launch': flop_launch},
            'train_mse_last_step': mse})
    if want('strong', a.no_strong):
        # configs[3] as written: global batch 4096 split over the ranks (strong scaling)
        n_loc = STRONG_GLOBAL // world
        m.set_weights(init_w)
        x, y = synth(n_loc, 4321 + rank, dev)
        st = max(3, a.steps // 4)
        dt, kms, _, _ = run_train(eng, m.optimizer, x, y, P, n_loc, n_loc * world, rank, world, st,
                                  min(2, a.warmup), dist)
        del x, y
        out['strong'] = {'workload': 'configs[3]: global batch %d images of 96x96 split over %d rank(s) '
                                     '(%d per rank), same model / optimizer' % (n_loc * world, world, n_loc),
                         'value': n_loc * world * st / dt, 'unit': 'images/sec', 'ms_per_step': dt * 1e3 / st,
                         'steps': st, 'scaling': 'strong', 'kernel_ms': kms}
    if rank == 0 and want('p1', a.no_p1) and world == 1:
        out['p1'] = bench_p1(keras, no_cpu=a.no_cpu)
    if rank == 0 and want('infer', a.no_infer):
        out['infer'] = bench_infer(hpe, dev, a.steps)
    if rank == 0 and want('train88', a.no_train88):
        out['train88'] = bench_train88(hpe, keras, dev, max(5, min(a.steps, 20)), 2)
    if rank == 0 and want('attn', a.no_attn):
        out['attn'] = bench_attn(dev, max(10, a.steps))
    if rank == 0 and want('blazeface', a.no_blaze):
        out['blazeface'] = bench_blazeface(dev, max(10, a.steps), a.no_cpu or world > 1)
    if rank == 0 and want('blazeface_b1', a.no_blaze):
        out['blazeface_b1'] = bench_blazeface_b1(dev, a.no_cpu or world > 1)
    if rank == 0 and world == 1 and want('train') and not a.no_cpu:
        cb = cpu_baseline((m.model_config, init_w))
        out['cpu_baseline'] = cb
        out['vs_cpu_baseline'] = out['value'] / cb['value']
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
