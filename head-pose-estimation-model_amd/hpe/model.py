"""keras.Model surface of the reference's regressors, executed by libhpe.so on the GPU.

The methods the reference calls are kept with their Keras 2.13 semantics:
  compile(optimizer, loss='mse', metrics=['mae'])                  train_96.py:105-109
  fit(x, y, epochs, batch_size, validation_data, callbacks, verbose)  train_96.py:175-183
  evaluate(x, y) -> [loss, mae]                                      train_96.py:186-187
  predict(x)                                                         test.py:34
  count_params(), to_json(), save(path), get_weights(), set_weights()  train_96.py:195-196
Loss is MSE over every output element plus the L2 regularisation terms, MAE the metric; epoch logs
are batch-size-weighted means as in Keras.  The whole dataset lives in HBM; each step is one
train-step kernel, one reduce, (one RCCL all-reduce when distributed) and one optimizer kernel.
"""
import json
import math
import os

import numpy as np

from . import layers as L
from . import optimizers as O
from . import random as hrandom
from .callbacks import Callback, History
from .parallel import all_reduce_grad, batch_slice

KERAS_VERSION = '2.13.1'


class Model:
    def __init__(self, inputs=None, outputs=None, name=None, _config=None, _weights=None):
        self.name = name or L.unique_name('model')
        if _config is not None:
            self._config = _config
            self._weights = dict(_weights)
            self._layer_order = None
        else:
            inputs = list(inputs) if isinstance(inputs, (list, tuple)) else [inputs]
            outputs = list(outputs) if isinstance(outputs, (list, tuple)) else [outputs]
            cfg, layers = L.model_config(self.name, inputs, outputs)
            self._config = cfg
            self._weights = {}
            for l in layers:
                for k, w in l.weights.items():
                    self._weights[l.name + '/' + k] = np.asarray(w, dtype=np.float32)
            self._out_shape = outputs[0].shape
        self._engine = None
        self.optimizer = None
        self.loss = None
        self.compiled_metrics = []
        self.stop_training = False
        self.history = None
        self._dist = None

    # -- structure ----------------------------------------------------------------------------
    @property
    def model_config(self):
        return {'class_name': 'Functional', 'config': self._config}

    def weight_keys(self):
        """Keras ``model.weights`` order: layer order, each layer's variables in creation order."""
        order = []
        rank = {'kernel': 0, 'depthwise_kernel': 0, 'pointwise_kernel': 1, 'bias': 2, 'gamma': 0,
                'beta': 1, 'moving_mean': 3, 'moving_variance': 4}
        sub = {'query': 0, 'key': 1, 'value': 2, 'attention_output': 3}

        def walk(cfg, pre):
            for l in cfg['layers']:
                if l['class_name'] == 'Functional':
                    walk(l['config'], pre + l['name'] + '/')
                    continue
                p = pre + l['name'] + '/'
                ks = [k for k in self._weights if k.startswith(p) and
                      k.count('/') <= p.count('/') + (1 if l['class_name'] == 'MultiHeadAttention' else 0)]
                ks.sort(key=lambda k: (sub.get(k[len(p):].split('/')[0], 0)
                                       if l['class_name'] == 'MultiHeadAttention' else 0,
                                       rank.get(k.rsplit('/', 1)[-1], 9)))
                order.extend(ks)
        walk(self._config, '')
        return order

    def count_params(self):
        return int(sum(int(np.prod(self._weights[k].shape)) for k in self.weight_keys()))

    def to_json(self, **kw):
        return json.dumps({'class_name': 'Functional', 'config': self._config,
                           'keras_version': KERAS_VERSION, 'backend': 'tensorflow'}, **kw)

    def summary(self, print_fn=print):
        print_fn('Model: "%s"' % self.name)
        for l in self._config['layers']:
            n = sum(int(np.prod(self._weights[k].shape)) for k in self._weights
                    if k.startswith(l['name'] + '/'))
            print_fn('  %-32s %-24s %8d' % (l['name'], l['class_name'], n))
        print_fn('Total params: %d' % self.count_params())

    # -- weights ------------------------------------------------------------------------------
    def _sync_from_device(self):
        if self._engine is not None:
            self._weights.update(self._engine.get_weights())

    def get_weights(self):
        self._sync_from_device()
        return [self._weights[k].copy() for k in self.weight_keys()]

    def set_weights(self, weights):
        keys = self.weight_keys()
        if isinstance(weights, dict):
            upd = {k: np.asarray(v, np.float32) for k, v in weights.items()}
        else:
            if len(weights) != len(keys):
                raise ValueError('set_weights: expected %d arrays, got %d' % (len(keys), len(weights)))
            upd = {k: np.asarray(w, np.float32) for k, w in zip(keys, weights)}
        for k, v in upd.items():
            if k not in self._weights:
                raise ValueError('unknown weight %s' % k)
            if v.shape != self._weights[k].shape:
                raise ValueError('weight %s: shape %s != %s' % (k, v.shape, self._weights[k].shape))
        self._weights.update(upd)
        if self._engine is not None:
            trainable = {k: v for k, v in upd.items() if k in self._engine.layout.param_index}
            self._engine.set_weights(trainable)

    def weights_dict(self):
        self._sync_from_device()
        return {k: self._weights[k].copy() for k in self.weight_keys()}

    # -- engine -------------------------------------------------------------------------------
    def _eng(self):
        if self._engine is None:
            from .engine import Engine
            self._engine = Engine(self.model_config, self._weights)
            self._apply_pending_opt(self._engine)
        return self._engine

    def compile(self, optimizer='rmsprop', loss=None, metrics=None, **kw):
        if loss not in ('mse', 'mean_squared_error', None):
            raise ValueError('only loss="mse" is on the hot path (train_96.py:51), got %r' % (loss,))
        self.optimizer = O.get(optimizer)
        self.loss = 'mse'
        self.compiled_metrics = list(metrics or [])
        for m in self.compiled_metrics:
            if m not in ('mae', 'mean_absolute_error'):
                raise ValueError('only metrics=["mae"] supported, got %r' % (m,))

    def distribute(self, group=None):
        """Data-parallel training over torch.distributed (RCCL): each rank takes a contiguous slice
        of every global batch, one all-reduce of the flat gradient per step."""
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            self._dist = (dist, group)
        return self

    # -- data helpers -------------------------------------------------------------------------
    def _rows(self, x):
        x = np.asarray(x, dtype=np.float32)
        if x.ndim == 2:
            n, c = x.shape
            P = 1
        elif x.ndim == 4:
            n, h, w, c = x.shape
            P = h * w
        else:
            raise ValueError('expected input of shape (N, H, W, C) or (N, C), got %s' % (x.shape,))
        return np.ascontiguousarray(x.reshape(n * P, c)), n, P, x.shape

    def _labels(self, y, n):
        y = np.asarray(y, dtype=np.float32)
        if y.size != n * 3:
            if y.ndim >= 2 and y.shape[0] == n:
                per = y.reshape(n, -1, 3)
                if np.all(per == per[:, :1, :]):
                    return np.ascontiguousarray(per[:, 0, :])
            raise ValueError('labels must be one (yaw, pitch, roll) triple per image; got %s'
                             % (y.shape,))
        return np.ascontiguousarray(y.reshape(n, 3))

    def _out_shape_for(self, xshape, n):
        outputs = self._config['output_layers']
        # spatial output unless the graph flattens (Flatten / Dense head on (C,))
        spatial = True
        names = {l['name']: l for l in self._config['layers']}
        for l in self._config['layers']:
            if l['class_name'] in ('Flatten',):
                spatial = False
            if l['class_name'] == 'GlobalAveragePooling2D':
                # a pooled output (create_model -> GAP), not the SE squeeze of the model input
                src = [t[0] for node in l.get('inbound_nodes') or [] for t in node]
                if not all(names.get(s, {}).get('class_name') == 'InputLayer' for s in src):
                    spatial = False
        if len(xshape) == 4 and spatial:
            return (n, xshape[1], xshape[2], 3)
        return (n, 3)

    # -- inference ----------------------------------------------------------------------------
    def predict(self, x, batch_size=None, verbose=0, **kw):
        import torch
        eng = self._eng()
        rows, n, P, shp = self._rows(x)
        xd = torch.from_numpy(rows).to(eng.device)
        y = eng.forward(xd, P)
        return y.cpu().numpy().reshape(self._out_shape_for(shp, n))

    def __call__(self, x, training=False):
        return self.predict(x)

    def _reg_loss(self):
        eng = self._eng()
        return float((eng.l2 * eng.params[:eng.n_train] ** 2).sum().item())

    def evaluate(self, x=None, y=None, batch_size=None, verbose='auto', return_dict=False, **kw):
        import torch
        eng = self._eng()
        rows, n, P, shp = self._rows(x)
        lab = self._labels(y, n)
        xd = torch.from_numpy(rows).to(eng.device)
        yd = torch.from_numpy(lab).to(eng.device)
        s = eng.loss_sums(xd, yd, P).cpu().numpy().astype(np.float64)
        cnt = n * P * 3
        loss = s[0] / cnt + self._reg_loss()
        mae = s[1] / cnt
        if verbose not in (0, 'auto') and verbose:
            print('loss: %.4f - mae: %.4f' % (loss, mae))
        if return_dict:
            return {'loss': loss, 'mae': mae}
        return [loss, mae] if self.compiled_metrics else loss

    # -- training -----------------------------------------------------------------------------
    def fit(self, x=None, y=None, batch_size=None, epochs=1, verbose='auto', callbacks=None,
            validation_data=None, shuffle=True, initial_epoch=0, **kw):
        import torch
        if self.optimizer is None:
            raise RuntimeError('You must compile your model before training/testing. Use '
                               '`model.compile(optimizer, loss)`.')
        eng = self._eng()
        rows, n, P, shp = self._rows(x)
        lab = self._labels(y, n)
        bs = int(batch_size or 32)
        xd = torch.from_numpy(rows).to(eng.device)
        yd = torch.from_numpy(lab).to(eng.device)
        if validation_data is not None:
            vrows, vn, vP, _ = self._rows(validation_data[0])
            vlab = self._labels(validation_data[1], vn)
            vxd = torch.from_numpy(vrows).to(eng.device)
            vyd = torch.from_numpy(vlab).to(eng.device)
        world, rank = 1, 0
        if self._dist is not None:
            dist, grp = self._dist
            world, rank = dist.get_world_size(grp), dist.get_rank(grp)
        hist = History()
        cbs = [hist] + list(callbacks or [])
        for cb in cbs:
            cb.set_model(self)
            cb.set_params({'epochs': epochs, 'steps': math.ceil(n / bs), 'verbose': verbose})
        self.stop_training = False
        for cb in cbs:
            cb.on_train_begin()
        rng = np.random.RandomState(hrandom.seed())
        steps = math.ceil(n / bs)
        og = eng.optim_grid()
        stats = torch.zeros((steps, 2 + og), dtype=torch.float32, device=eng.device)
        # the reference's regime (P = 1, create_model family, one rank): the whole epoch is one
        # launch (csrc/hpe_fit.hip); otherwise one train_step + reduce + optimizer per step
        fused = eng.fit_epoch_supported(bs, P, world)
        self._last_fit_fused = fused
        # one bound on the resident rows per call: below the fp16 split's data range (64) the
        # per-step launches skip their exact-fp32 twin (csrc/hpe_mlp2.hip launch_pair)
        x_bound = 0.0 if fused or not xd.numel() else max(-float(xd.amin().item()), float(xd.amax().item()))
        if not np.isfinite(x_bound):
            x_bound = 0.0
        if fused:  # [sse, sae, per-wave regularisation shares of the 4 G waves]
            stats = torch.zeros((steps, 2 + 4 * eng.fit_groups()), dtype=torch.float32, device=eng.device)
        for epoch in range(initial_epoch, epochs):
            for cb in cbs:
                cb.on_epoch_begin(epoch)
            perm = rng.permutation(n) if shuffle else np.arange(n)
            idx = torch.from_numpy(perm.astype(np.int32)).to(eng.device)
            nbs = [min(n, (s + 1) * bs) - s * bs for s in range(steps)]
            if fused:
                stats.zero_()
                if eng.fit_epoch(self.optimizer, xd, yd, idx, bs, stats, hrandom.dropout_seed(0)) is None:
                    # the epoch launch timed out and was rolled back: this and later epochs per step
                    fused = self._last_fit_fused = False
                    stats = torch.zeros((steps, 2 + og), dtype=torch.float32, device=eng.device)
            # per-step path: the whole step loop in one C call (hpe_fit_steps; under data parallelism
            # hpe_fit_steps_dp with a per-step all-reduce hook: the same launches as the loop below,
            # without a Python round trip per step); HPE_FIT_STEPS=0 keeps the Python loop
            c_steps = not fused and os.environ.get('HPE_FIT_STEPS', '1') != '0'
            if c_steps:
                # (HPE_FIT_DP_ONE_RANK=1: the data-parallel step loop on a one-rank group, for tests)
                dp = world > 1 or os.environ.get('HPE_FIT_DP_ONE_RANK') == '1'
                eng.fit_steps(self.optimizer, xd, yd, idx, bs, stats, hrandom.dropout_seed(0), x_bound, P,
                              dist=self._dist if dp else None)
            for s in range(0 if fused or c_steps else steps):
                b0, b1 = s * bs, min(n, (s + 1) * bs)
                nb = b1 - b0
                r0, r1 = batch_slice(b0, b1, rank, world)   # this rank's share of the batch
                seed = hrandom.dropout_seed(eng.iterations + 1)
                if r1 > r0:
                    eng.gradient(xd, yd, P, idx[r0:r1], r1 - r0, 1.0 / (nb * P * 3), seed,
                                 img_off=r0 - b0, defer_reduce=world == 1, x_bound=x_bound)
                else:
                    eng.grad.zero_()
                if world > 1:
                    all_reduce_grad(eng.grad, self._dist[1])
                eng.optimizer_step(self.optimizer, stats[s])
            st = stats.cpu().numpy().astype(np.float64)
            nbs = np.asarray(nbs, dtype=np.float64)
            loss = float((st[:, 0].sum() / (P * 3) + (nbs * st[:, 2:].sum(axis=1)).sum()) / n)
            mae = float(st[:, 1].sum() / (n * P * 3))
            logs = {'loss': loss, 'mae': mae}
            if validation_data is not None:
                vs = eng.loss_sums(vxd, vyd, vP).cpu().numpy().astype(np.float64)
                vc = vn * vP * 3
                logs['val_loss'] = float(vs[0] / vc + self._reg_loss())
                logs['val_mae'] = float(vs[1] / vc)
            self.optimizer.iterations = eng.iterations
            if verbose and verbose != 0:
                print('Epoch %d/%d - ' % (epoch + 1, epochs) +
                      ' - '.join('%s: %.4f' % (k, v) for k, v in logs.items()))
            for cb in cbs:
                cb.on_epoch_end(epoch, logs)
            if self.stop_training:
                break
        for cb in cbs:
            cb.on_train_end()
        self.history = hist
        hist.model = self
        return hist

    # -- persistence --------------------------------------------------------------------------
    def _h5_layer_weights(self):
        """[(layer_name, [(keras weight name, array)])] in model.layers order, as Keras's
        save_weights_to_hdf5_group lays them out (a nested Functional layer's variables keep their
        own names: 'conv2d/kernel:0' under group 'model')."""
        keys = self.weight_keys()
        out = []
        for l in self._config['layers']:
            ln = l['name']
            ws = []
            for k in keys:
                if not k.startswith(ln + '/'):
                    continue
                wn = k[len(ln) + 1:] if l['class_name'] == 'Functional' else k
                ws.append((wn + ':0', self._weights[k]))
            out.append((ln, ws))
        return out

    def _training_config(self):
        if self.optimizer is None:
            return None
        o = self.optimizer
        f32 = lambda v: float(np.float32(v))  # noqa: E731  (Keras stores the variables' float32 values)
        cfg = {'name': o.name, 'learning_rate': f32(o.learning_rate), 'decay': 0.0}
        if o.kind == 'sgd':
            cfg.update(momentum=0.0, nesterov=False)
        else:
            cfg.update(beta_1=f32(o.beta_1), beta_2=f32(o.beta_2), epsilon=o.epsilon)
            if o.kind == 'adam':
                cfg['amsgrad'] = False
        return {'loss': 'mse',
                'metrics': [[{'class_name': 'MeanMetricWrapper',
                              'config': {'name': 'mae', 'dtype': 'float32', 'fn': 'mean_absolute_error'}}]]
                if self.compiled_metrics else None,
                'weighted_metrics': None, 'loss_weights': None,
                'optimizer_config': {'class_name': type(o).__name__, 'config': cfg}}

    def _optimizer_state(self):
        """Legacy Keras optimizer variables [(name, array)]: '<Opt>/iter:0', then every
        trainable weight's m, then every v (Model-96/Trained-Models-96/*.h5 'optimizer_weights')."""
        if self.optimizer is None:
            return None
        nm = type(self.optimizer).__name__
        eng = self._engine
        it = int(eng.iterations) if eng is not None else int(getattr(self, '_pending_opt', {}).get('iter', 0))
        out = [('%s/iter:0' % nm, np.asarray(it, np.int64))]
        if self.optimizer.kind == 'sgd':
            return out
        if eng is not None and eng.m is not None:
            m, v = eng.m.cpu().numpy(), eng.v.cpu().numpy()
            idx = eng.layout.param_index
            keys = [k for k in self.weight_keys() if k in idx]
            get = lambda a, k: a[idx[k][0]:idx[k][0] + int(np.prod(idx[k][1]))].reshape(idx[k][1])  # noqa: E731
        else:
            pend = getattr(self, '_pending_opt', None)
            if not pend or not pend.get('m'):
                return out
            keys = [k for k in self.weight_keys() if k in pend['m']]
            m, v = pend['m'], pend['v']
            get = lambda a, k: a[k]  # noqa: E731
        out += [('%s/%s/m:0' % (nm, k), get(m, k)) for k in keys]
        out += [('%s/%s/v:0' % (nm, k), get(v, k)) for k in keys]
        return out

    def save(self, filepath, include_optimizer=True, **kw):
        """``.h5`` / ``.hdf5``: a Keras 2.13 legacy HDF5 checkpoint (hpe.h5io.write_keras_h5), the
        format ModelCheckpoint writes at Model-96/train_96.py:153-158 and Model-88/train_88.py:335;
        any other name: the same content in an npz container."""
        self._sync_from_device()
        d = os.path.dirname(str(filepath))
        if d:
            os.makedirs(d, exist_ok=True)
        if str(filepath).endswith(('.h5', '.hdf5')):
            from . import h5io
            h5io.write_keras_h5(str(filepath), self.model_config, self._h5_layer_weights(),
                                training_config=self._training_config(),
                                optimizer_weights=self._optimizer_state() if include_optimizer else None,
                                keras_version=KERAS_VERSION)
            return
        arrs = {'__model_config__': np.frombuffer(json.dumps(self.model_config).encode(), np.uint8),
                '__keras_version__': np.frombuffer(KERAS_VERSION.encode(), np.uint8)}
        for k in self.weight_keys():
            arrs['w/' + k] = self._weights[k]
        for n, a in (self._optimizer_state() or []) if include_optimizer else []:
            arrs['o/' + n[:-2]] = a
        with open(filepath, 'wb') as fh:
            np.savez(fh, **arrs)

    def _set_optimizer_state(self, opt_weights):
        """Stage a legacy optimizer state ({'Adam/iter': n, 'Adam/<key>/m': arr, ...}) to be
        loaded into the device buffers when the engine is created (Keras restores it on
        load_model(compile=True))."""
        pend = {'iter': 0, 'm': {}, 'v': {}}
        for n, a in opt_weights.items():
            parts = n.split('/')
            if parts[-1] == 'iter':
                pend['iter'] = int(np.asarray(a))
            elif parts[-1] in ('m', 'v'):
                pend[parts[-1]]['/'.join(parts[1:-1])] = np.asarray(a, np.float32)
        self._pending_opt = pend
        if self._engine is not None:
            self._apply_pending_opt(self._engine)

    def _apply_pending_opt(self, eng):
        pend = getattr(self, '_pending_opt', None)
        if not pend:
            return
        import torch
        eng.iterations = pend['iter']
        if pend['m']:
            m = np.zeros(eng.n_train, np.float32)
            v = np.zeros(eng.n_train, np.float32)
            for k, (o, shp) in eng.layout.param_index.items():
                n = int(np.prod(shp))
                if k in pend['m']:
                    m[o:o + n] = pend['m'][k].ravel()
                    v[o:o + n] = pend['v'][k].ravel()
            eng.m = torch.from_numpy(m).to(eng.device)
            eng.v = torch.from_numpy(v).to(eng.device)
        self._pending_opt = None

    def load_weights(self, filepath):
        m = load_model(filepath)
        self.set_weights(m.weights_dict())


def model_from_config(model_config, weights, name=None):
    cfg = model_config.get('config', model_config)
    from . import blazeface
    if blazeface.is_blazeface(cfg):
        return blazeface.UnifiedModel({'class_name': 'Functional', 'config': cfg}, weights, name=name)
    return Model(name=name or cfg.get('name'), _config=cfg, _weights=weights)


def _compile_from(model, training_config, opt_state):
    """Keras load_model(compile=True): re-create the optimizer from training_config (class and
    hyper-parameters) and restore its state (iterations, m, v)."""
    if not training_config or not isinstance(model, Model):
        return model
    oc = training_config.get('optimizer_config') or {}
    cls = {'SGD': O.SGD, 'Adam': O.Adam, 'Adamax': O.Adamax}.get(oc.get('class_name'))
    if cls is None:
        return model
    c = dict(oc.get('config', {}))
    kw = {k: c[k] for k in ('learning_rate', 'beta_1', 'beta_2', 'epsilon', 'name') if k in c}
    model.compile(optimizer=cls(**kw), loss='mse',
                  metrics=['mae'] if training_config.get('metrics') else None)
    if opt_state:
        model._set_optimizer_state(opt_state)
    return model


def load_model(filepath, compile=True, **kw):
    """Load a model saved by Model.save, a converted fixture (<id>.json + <id>.npz), or a Keras
    ``.h5`` file (via hpe.h5io); with compile=True the optimizer and its state come back too
    (test.py:31 loads the reference's checkpoints this way)."""
    p = str(filepath)
    if p.endswith('.json') or (not os.path.exists(p) and os.path.exists(p + '.json')):
        base = p[:-5] if p.endswith('.json') else p
        with open(base + '.json') as fh:
            meta = json.load(fh)
        w = dict(np.load(base + '.npz'))
        return model_from_config(meta['model_config'], w)
    if not os.path.exists(p):
        raise FileNotFoundError('No file or directory found at %s' % p)
    with open(p, 'rb') as fh:
        magic = fh.read(8)
    if magic.startswith(b'\x89HDF'):
        from . import h5io
        mc, w, opt = h5io.read_keras_h5(p, with_optimizer=True)
        m = model_from_config(mc, w)
        return _compile_from(m, h5io.read_training_config(p), opt) if compile else m
    z = np.load(p, allow_pickle=False)
    mc = json.loads(bytes(z['__model_config__']).decode())
    w = {k[2:]: z[k] for k in z.files if k.startswith('w/')}
    return model_from_config(mc, w)
