"""CPU restatement of the reference's Keras 2.13 layer / loss / optimizer semantics.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): the checker the HIP path is compared with, and
the ``cpu_baseline`` leg of bench.py.  Written from the Keras layer semantics the reference calls
(TF/Keras 2.13 itself is absent here); every public function cites the reference call site it
restates.  Gradients come from torch.autograd, the same reverse-mode autodiff Keras' ``fit`` uses
(``Model-96/train_96.py:175``) — independent of the hand-derived HIP backward it checks.

Default dtype float64; ``dtype=torch.float32`` gives the fp32 restatement timed as CPU baseline.
"""
import json
import math

import numpy as np
import torch
import torch.nn.functional as F

# ----------------------------------------------------------------------------------------------
# activations  (Conv2D/Dense ``activation=`` strings: train_96.py:76, train_88.py:79,
# attention_model.py:36-37,61,77; checkpoint-only strings listed in SURVEY.md §2 row 2)
# ----------------------------------------------------------------------------------------------
SELU_ALPHA = 1.6732632423543772848170429916717
SELU_SCALE = 1.0507009873554804934193349852946


def activation(name, x):
    if name in (None, 'linear'):
        return x
    if name == 'tanh':
        return torch.tanh(x)
    if name == 'relu':
        return torch.relu(x)
    if name == 'softsign':
        return x / (1.0 + x.abs())
    if name == 'sigmoid':
        return torch.sigmoid(x)
    if name == 'elu':
        return torch.where(x > 0, x, torch.expm1(x))
    if name == 'selu':
        return SELU_SCALE * torch.where(x > 0, x, SELU_ALPHA * torch.expm1(x))
    if name == 'swish':
        return x * torch.sigmoid(x)
    if name == 'softplus':
        return F.softplus(x)
    if name == 'leaky_relu':  # tf.nn.leaky_relu default alpha (only Model-88 yu8tzyf8.h5)
        return torch.where(x > 0, x, 0.2 * x)
    raise ValueError('Unknown activation function: %r' % (name,))


# ----------------------------------------------------------------------------------------------
# SpatialDropout2D mask (train_96.py:82,94; train_88.py:84).  TF's RNG cannot be reproduced
# (SURVEY.md §7 hard part iii); the build's counter hash is restated here so a dropout>0
# training step can be compared mask-for-mask.  keep(b, c) broadcast over H, W; scale 1/(1-rate).
# ----------------------------------------------------------------------------------------------
M64 = (1 << 64) - 1


def _mix64(z):
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def dropout_hash(seed, drop_id, image, chan):
    """uint32 hash of (seed, dropout-layer ordinal, image index in batch, channel): a 64-bit
    splitmix of (seed, ordinal, image), then a 32-bit murmur3 finaliser of (its high word, channel)
    (csrc/hpe_common.h drop_base / drop_mix)."""
    with np.errstate(over='ignore'):
        image = np.asarray(image, dtype=np.uint64)
        chan = np.asarray(chan, dtype=np.uint64)
        x = np.uint64((int(seed) + 0x9E3779B97F4A7C15 * (1 + int(drop_id))) & M64)
        x = x ^ (image * np.uint64(0xBF58476D1CE4E5B9))
        base = (_mix64(x) >> np.uint64(32)).astype(np.uint64)
        m32 = np.uint64(0xFFFFFFFF)
        h = base ^ ((chan * np.uint64(0x9E3779B9)) & m32)
        h = h ^ (h >> np.uint64(16))
        h = (h * np.uint64(0x85EBCA6B)) & m32
        h = h ^ (h >> np.uint64(13))
        h = (h * np.uint64(0xC2B2AE35)) & m32
        h = h ^ (h >> np.uint64(16))
        return h.astype(np.uint32)


def dropout_threshold(rate):
    return min(int(math.floor(float(rate) * 4294967296.0)), 4294967295)


def dropout_mask(seed, drop_id, n_images, channels, rate, image_offset=0):
    """(n_images, channels) float mask: 0 or 1/(1-rate)."""
    img = np.arange(image_offset, image_offset + n_images, dtype=np.uint64)[:, None]
    ch = np.arange(channels, dtype=np.uint64)[None, :]
    keep = dropout_hash(seed, drop_id, img, ch) >= np.uint32(dropout_threshold(rate))
    return keep.astype(np.float64) * (1.0 / (1.0 - float(np.float32(rate))))


# ----------------------------------------------------------------------------------------------
# spatial helpers: TF 'same' padding (asymmetric for stride 2)
# ----------------------------------------------------------------------------------------------
def _same_pads(n, k, s):
    out = -(-n // s)
    tot = max((out - 1) * s + k - n, 0)
    return tot // 2, tot - tot // 2


def _pad_same(x_nchw, kh, kw, sh, sw, value=0.0):
    pt, pb = _same_pads(x_nchw.shape[2], kh, sh)
    pl, pr = _same_pads(x_nchw.shape[3], kw, sw)
    return F.pad(x_nchw, (pl, pr, pt, pb), value=value)


def _to_nchw(x):
    return x.permute(0, 3, 1, 2)


def _to_nhwc(x):
    return x.permute(0, 2, 3, 1)


def _reg_coeff(reg):
    if not reg:
        return 0.0
    cfg = reg.get('config', {})
    if reg.get('class_name') in ('L2', 'L1L2'):
        return float(cfg.get('l2', 0.0))
    return 0.0


# ----------------------------------------------------------------------------------------------
# graph executor over a Keras ``model_config`` (the JSON every .h5 stores; Model-88/model.json)
# ----------------------------------------------------------------------------------------------
class Graph:
    """Forward (and autograd backward) of a Keras Functional ``model_config``.

    Layer semantics restated (reference call sites):
      Conv2D 1x1 / kxk 'same'|'valid'   train_96.py:72-92, train_88.py:76-140, attention_model.py:77
      Conv2DTranspose 3x3 s1 'same'     checkpoint cshlz666.h5 only
      SeparableConv2D (dw then pw)      checkpoint o6e5xpan.h5 etc.
      DepthwiseConv2D, MaxPooling2D, ReLU, Pad/Reshape TFOpLayers   BlazeFace, blazeFaceDetectorH5.py:272
      Dense                              attention_model.py:36-37,58-59
      SpatialDropout2D                   train_96.py:82,94
      Add/Average/Multiply/Activation    attention_model.py:38,56,60,148-149
      GlobalAveragePooling2D/Reshape     attention_model.py:35,37
      Lambda (flatten HW / reshape back) attention_model.py:43-50,66-72  (bytecode never run)
      MultiHeadAttention                 attention_model.py:52-55
      LayerNormalization                 attention_model.py:57,61
      BatchNormalization (inference)     checkpoint dkgzatqk.h5 etc.
      nested Functional                  JoinModels.py:43-44,65-66 (unified models)
    """

    def __init__(self, model_config, weights, dtype=torch.float64, prefix=''):
        mc = model_config.get('config', model_config)
        self.name = mc.get('name', 'model')
        self.dtype = dtype
        self.layers = {l.get('name', l['config'].get('name')): l for l in mc['layers']}
        self.order = [l['name'] for l in mc['layers']]
        self.inputs = [t[0] for t in mc['input_layers']]
        self.outputs = [t[0] for t in mc['output_layers']]
        self.params = {}
        self.l2 = {}
        self.trainable = []
        self.sub = {}
        self.drop_ids = {}
        for l in mc['layers']:
            if l['class_name'] == 'SpatialDropout2D':
                self.drop_ids[l['name']] = len(self.drop_ids)
        for l in mc['layers']:
            name, cls, cfg = l['name'], l['class_name'], l['config']
            if cls == 'Functional':
                self.sub[name] = Graph(cfg, weights, dtype, prefix + name + '/')
                for k, v in self.sub[name].params.items():
                    self.params[k] = v
                    self.l2[k] = self.sub[name].l2[k]
                self.trainable += self.sub[name].trainable
                continue
            keys = [k for k in weights if k.startswith(prefix + name + '/')
                    and k.count('/') - prefix.count('/') >= 1]
            for k in self._weight_order(cls, name, prefix, keys):
                t = torch.tensor(np.asarray(weights[k]), dtype=dtype)
                self.params[k] = t
                base = k.rsplit('/', 1)[-1]
                if base in ('kernel', 'depthwise_kernel', 'pointwise_kernel'):
                    self.l2[k] = _reg_coeff(cfg.get('kernel_regularizer'))
                elif base == 'bias' and cls != 'MultiHeadAttention':
                    self.l2[k] = _reg_coeff(cfg.get('bias_regularizer'))
                else:
                    self.l2[k] = 0.0
                if base not in ('moving_mean', 'moving_variance'):
                    self.trainable.append(k)

    @staticmethod
    def _weight_order(cls, name, prefix, keys):
        # Keras trainable_weights order: kernel before bias; MHA q,k,v,o
        rank = {'kernel': 0, 'depthwise_kernel': 0, 'pointwise_kernel': 1, 'bias': 2, 'gamma': 0,
                'beta': 1, 'moving_mean': 3, 'moving_variance': 4}
        sub = {'query': 0, 'key': 1, 'value': 2, 'attention_output': 3}

        def key(k):
            parts = k[len(prefix):].split('/')
            return (sub.get(parts[1], 0) if len(parts) > 2 else 0, rank.get(parts[-1], 9))
        return sorted(keys, key=key)

    def p(self, name, prefix=''):
        return self.params[prefix + name]

    # ------------------------------------------------------------------------------------------
    def forward(self, x, training=False, drop_seed=0, image_offset=0, masks=None, _prefix=''):
        """Run the graph.  ``x``: numpy/torch (B,H,W,C) or (B,C).  Returns tensor or list."""
        if not torch.is_tensor(x):
            x = torch.tensor(np.asarray(x), dtype=self.dtype)
        cache = {self.inputs[0]: x}
        self._training, self._seed, self._off, self._masks = training, drop_seed, image_offset, masks

        def ev(name):
            if name in cache:
                return cache[name]
            l = self.layers[name]
            ins = [ev(t[0]) for node in l['inbound_nodes'] for t in node] if l['inbound_nodes'] else []
            kw = {}
            for node in (l['inbound_nodes'] or []):
                for t in node:
                    for kname, ref in (t[3] if len(t) > 3 else {}).items():
                        if isinstance(ref, list) and ref and isinstance(ref[0], str):
                            kw[kname] = ev(ref[0])
            self._kw = kw
            out = self._layer(l, ins, _prefix)
            cache[name] = out
            return out
        outs = [ev(o) for o in self.outputs]
        return outs[0] if len(outs) == 1 else outs

    def _layer(self, l, ins, prefix):
        cls, cfg, name = l['class_name'], l['config'], l['name']
        P = lambda w: self.params[prefix + name + '/' + w]
        x = ins[0] if ins else None
        if cls == 'Functional':
            g = self.sub[name]
            return g.forward(x, self._training, self._seed, self._off, self._masks,
                             _prefix=prefix + name + '/')
        if cls == 'InputLayer':
            return x
        if cls in ('Conv2D', 'Conv2DTranspose', 'SeparableConv2D', 'DepthwiseConv2D'):
            kh, kw = cfg['kernel_size']
            sh, sw = cfg['strides']
            if tuple(cfg.get('dilation_rate', (1, 1))) != (1, 1):
                raise ValueError('dilation_rate != 1 not supported')
            xn = _to_nchw(x)
            if cls == 'DepthwiseConv2D' or cls == 'SeparableConv2D':
                dk = P('depthwise_kernel')  # (kh,kw,C,mult)
                C, mult = dk.shape[2], dk.shape[3]
                w = dk.permute(2, 3, 0, 1).reshape(C * mult, 1, kh, kw)
                if cfg['padding'] == 'same':
                    xn = _pad_same(xn, kh, kw, sh, sw)
                xn = F.conv2d(xn, w, stride=(sh, sw), groups=C)
                if cls == 'SeparableConv2D':
                    pk = P('pointwise_kernel')  # (1,1,C*mult,F)
                    xn = F.conv2d(xn, pk.permute(3, 2, 0, 1))
            elif cls == 'Conv2D':
                k = P('kernel')
                if cfg['padding'] == 'same':
                    xn = _pad_same(xn, kh, kw, sh, sw)
                xn = F.conv2d(xn, k.permute(3, 2, 0, 1), stride=(sh, sw))
            else:  # Conv2DTranspose, stride 1 'same' odd kernel only
                if (sh, sw) != (1, 1) or cfg['padding'] != 'same' or kh % 2 == 0:
                    raise ValueError('Conv2DTranspose: only stride 1, odd kernel, same padding')
                k = P('kernel')  # (kh,kw,out,in)
                xn = F.conv_transpose2d(xn, k.permute(3, 2, 0, 1), padding=(kh // 2, kw // 2))
            y = _to_nhwc(xn)
            if cfg.get('use_bias', True):
                y = y + P('bias')
            return activation(cfg.get('activation'), y)
        if cls == 'Dense':
            y = torch.matmul(x, P('kernel'))
            if cfg.get('use_bias', True):
                y = y + P('bias')
            return activation(cfg.get('activation'), y)
        if cls == 'Activation':
            return activation(cfg['activation'], x)
        if cls == 'ReLU':
            if cfg.get('max_value') is not None or cfg.get('negative_slope', 0) or cfg.get('threshold', 0):
                raise ValueError('ReLU: only plain relu supported')
            return torch.relu(x)
        if cls == 'SpatialDropout2D':
            if not self._training or float(cfg['rate']) == 0.0:
                return x
            did = self.drop_ids[name]
            if self._masks is not None and (prefix + name) in self._masks:
                m = self._masks[prefix + name]
            else:
                m = dropout_mask(self._seed, did, x.shape[0], x.shape[-1], cfg['rate'], self._off)
            m = torch.as_tensor(m, dtype=x.dtype).reshape(x.shape[0], *([1] * (x.dim() - 2)), x.shape[-1])
            return x * m
        if cls == 'Add':
            y = ins[0]
            for t in ins[1:]:
                y = y + t
            return y
        if cls == 'Average':
            y = ins[0]
            for t in ins[1:]:
                y = y + t
            return y / len(ins)
        if cls == 'Multiply':
            y = ins[0]
            for t in ins[1:]:
                y = y * t
            return y
        if cls == 'Flatten':
            return x.reshape(x.shape[0], -1)
        if cls == 'Reshape':
            return x.reshape(x.shape[0], *cfg['target_shape'])
        if cls == 'GlobalAveragePooling2D':
            return x.mean(dim=(1, 2), keepdim=bool(cfg.get('keepdims', False)))
        if cls == 'MaxPooling2D':
            ph, pw = cfg['pool_size']
            sh, sw = cfg['strides']
            xn = _to_nchw(x)
            if cfg['padding'] == 'same':
                xn = _pad_same(xn, ph, pw, sh, sw, value=-math.inf)
            return _to_nhwc(F.max_pool2d(xn, (ph, pw), (sh, sw)))
        if cls == 'Lambda':
            # attention_model.py:43-50 (flatten H,W) and :66-72 (reshape back to orig)
            if len(ins) == 1:
                B, H, W, C = x.shape
                return x.reshape(B, H * W, C)
            t, orig = ins
            return t.reshape(orig.shape[0], orig.shape[1], orig.shape[2], t.shape[-1])
        if cls == 'TensorFlowOpLayer':
            op = cfg['node_def']['op']
            const = cfg['constants']
            if op == 'Pad':
                pads = const['1']
                fp = []
                for a, b in reversed(pads):
                    fp += [a, b]
                return F.pad(x, fp)
            if op == 'Reshape':
                shp = list(const['1'])
                return x.reshape(x.shape[0], *shp[1:])
            raise ValueError('TensorFlowOpLayer op %r not supported' % op)
        if cls == 'LayerNormalization':
            eps = float(cfg['epsilon'])
            mu = x.mean(dim=-1, keepdim=True)
            var = ((x - mu) ** 2).mean(dim=-1, keepdim=True)
            y = (x - mu) * torch.rsqrt(var + eps)
            if cfg.get('scale', True):
                y = y * P('gamma')
            if cfg.get('center', True):
                y = y + P('beta')
            return y
        if cls == 'BatchNormalization':
            if self._training:
                raise ValueError('BatchNormalization training mode is not on the hot path')
            eps = float(cfg['epsilon'])
            inv = torch.rsqrt(P('moving_variance') + eps)
            if cfg.get('scale', True):
                inv = inv * P('gamma')
            y = (x - P('moving_mean')) * inv
            if cfg.get('center', True):
                y = y + P('beta')
            return y
        if cls == 'MultiHeadAttention':
            q_in = ins[0]
            v_in = ins[1] if len(ins) > 1 else self._kw.get('value', ins[0])
            k_in = ins[2] if len(ins) > 2 else self._kw.get('key', v_in)
            if cfg.get('attention_axes') not in (None, [1]):
                raise ValueError('MultiHeadAttention: attention over axis 1 only')
            dk = cfg['key_dim']
            q = torch.einsum('btc,chd->bthd', q_in, P('query/kernel')) + P('query/bias')
            k = torch.einsum('btc,chd->bthd', k_in, P('key/kernel')) + P('key/bias')
            v = torch.einsum('btc,chd->bthd', v_in, P('value/kernel')) + P('value/bias')
            q = q * (1.0 / math.sqrt(float(dk)))
            s = torch.einsum('bshd,bthd->bhts', k, q)  # (B, h, Tq, Tk)
            a = torch.softmax(s, dim=-1)
            o = torch.einsum('bhts,bshd->bthd', a, v)
            return torch.einsum('bthd,hdc->btc', o, P('attention_output/kernel')) + P('attention_output/bias')
        raise ValueError('Unknown layer: %s' % cls)

    def regularization(self):
        tot = None
        for k, c in self.l2.items():
            if c:
                t = c * (self.params[k] ** 2).sum()
                tot = t if tot is None else tot + t
        return tot


def layer_inbound(l):
    return [t[0] for node in l['inbound_nodes'] for t in node] if l['inbound_nodes'] else []


# ----------------------------------------------------------------------------------------------
# losses / metrics  (compile(loss='mse', metrics=['mae']): train_96.py:51-52,105-109)
# ----------------------------------------------------------------------------------------------
def mse(y_true, y_pred):
    return ((y_pred - y_true) ** 2).mean()


def mae(y_true, y_pred):
    return (y_pred - y_true).abs().mean()


# ----------------------------------------------------------------------------------------------
# optimizers: Keras LEGACY formulas (checkpoint state names 'Adam/<layer>/kernel/m', 'Adam/iter';
# train_96.py:99-103, train_88.py:323)
# ----------------------------------------------------------------------------------------------
class LegacyOptimizer:
    def __init__(self, kind, learning_rate, beta_1=0.9, beta_2=0.999, epsilon=1e-7):
        self.kind = kind.lower()
        self.lr, self.b1, self.b2, self.eps = learning_rate, beta_1, beta_2, epsilon
        self.iter = 0
        self.m, self.v = {}, {}

    def apply(self, params, grads):
        t = self.iter + 1
        with torch.no_grad():
            for k, g in grads.items():
                w = params[k]
                if self.kind == 'sgd':
                    w -= self.lr * g
                    continue
                m = self.m.setdefault(k, torch.zeros_like(w))
                v = self.v.setdefault(k, torch.zeros_like(w))
                # TF ApplyAdam / ApplyAdaMax functors (what Keras' legacy optimizers dispatch to)
                m.add_((g - m) * (1 - self.b1))
                if self.kind == 'adam':
                    v.add_((g * g - v) * (1 - self.b2))
                    alpha = self.lr * math.sqrt(1 - self.b2 ** t) / (1 - self.b1 ** t)
                    w -= (m * alpha) / (v.sqrt() + self.eps)
                elif self.kind == 'adamax':
                    torch.maximum(self.b2 * v, g.abs(), out=v)
                    w -= (self.lr / (1 - self.b1 ** t)) * (m / (v + self.eps))
                else:
                    raise ValueError('unknown optimizer %r' % self.kind)
        self.iter = t


def train_step(graph, opt, x, y, drop_seed=0, masks=None, image_offset=0):
    """One ``fit`` step (train_96.py:175): fwd (training) + mse + L2 + autodiff + optimizer.

    Returns (total_loss, mae) as floats computed on the pre-update weights, like Keras' logs."""
    params = graph.params
    tr = [k for k in graph.trainable]
    for k in tr:
        params[k].requires_grad_(True)
    if not torch.is_tensor(y):
        y = torch.tensor(np.asarray(y), dtype=graph.dtype)
    p = graph.forward(x, training=True, drop_seed=drop_seed, masks=masks, image_offset=image_offset)
    yb = y.reshape(y.shape[0], *([1] * (p.dim() - 2)), y.shape[-1]).expand_as(p)
    loss = mse(yb, p)
    reg = graph.regularization()
    total = loss + reg if reg is not None else loss
    gr = torch.autograd.grad(total, [params[k] for k in tr], allow_unused=True)
    grads = {k: (g if g is not None else torch.zeros_like(params[k])) for k, g in zip(tr, gr)}
    m = mae(yb, p).item()
    for k in tr:
        params[k].requires_grad_(False)
    opt.apply(params, grads)
    return float(total.item()), m, grads


def gradients(graph, x, y, drop_seed=0, masks=None):
    tr = list(graph.trainable)
    for k in tr:
        graph.params[k].requires_grad_(True)
    y = torch.tensor(np.asarray(y), dtype=graph.dtype) if not torch.is_tensor(y) else y
    p = graph.forward(x, training=True, drop_seed=drop_seed, masks=masks)
    yb = y.reshape(y.shape[0], *([1] * (p.dim() - 2)), y.shape[-1]).expand_as(p)
    loss = mse(yb, p)
    reg = graph.regularization()
    total = loss + reg if reg is not None else loss
    gr = torch.autograd.grad(total, [graph.params[k] for k in tr], allow_unused=True)
    for k in tr:
        graph.params[k].requires_grad_(False)
    return {k: (g if g is not None else torch.zeros_like(graph.params[k])).detach()
            for k, g in zip(tr, gr)}, float(total.item()), float(mae(yb, p).item())


# ----------------------------------------------------------------------------------------------
# data / evaluation
# ----------------------------------------------------------------------------------------------
def split_indices(n, test_size=0.2, random_state=42):
    """sklearn train_test_split(test_size=.2, random_state=42) index split (train_96.py:142-146,
    train_88.py:301-305): perm = RandomState(42).permutation(n); test = perm[:ceil(.2n)]."""
    perm = np.random.RandomState(random_state).permutation(n)
    n_test = int(math.ceil(test_size * n))
    return perm[n_test:], perm[:n_test]


def evaluate_head_pose(predictions, ground_truth):
    """Metric block of evaluate_head_pose_model (Model-96/test.py:41-54)."""
    predictions = np.asarray(predictions, dtype=np.float64).reshape(-1, 3)
    ground_truth = np.asarray(ground_truth, dtype=np.float64).reshape(-1, 3)
    mae_pa = np.mean(np.abs(predictions - ground_truth), axis=0)
    mse_pa = np.mean(np.square(predictions - ground_truth), axis=0)
    names = ['yaw', 'pitch', 'roll']
    out = {'MAE': {names[i]: float(mae_pa[i]) for i in range(3)},
           'MSE': {names[i]: float(mse_pa[i]) for i in range(3)}}
    out['MAE']['average'] = float(np.mean(mae_pa))
    out['MSE']['average'] = float(np.mean(mse_pa))
    return out


def load_fixture(path_no_ext, dtype=torch.float64):
    with open(path_no_ext + '.json') as fh:
        meta = json.load(fh)
    w = dict(np.load(path_no_ext + '.npz'))
    return Graph(meta['model_config'], w, dtype=dtype), meta
