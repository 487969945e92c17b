"""Lower a Keras ``model_config`` (+ weights) to a row program for libhpe's persistent kernel.

The reference's regressors (Model-96/train_96.py:65-110, Model-88/train_88.py:66-253,
Model-88/attention_model.py:16-169, and the 684 checkpoint graphs) are per-position DAGs: every
Conv2D in them has a 1x1 kernel (or is evaluated on 1x1 inputs), so each spatial position is an
independent row.  This module turns such a graph into the op list documented in
csrc/hpe_prog.h: forward ops with fused epilogues (activation + SpatialDropout), and — for
training — the loss, the reverse-mode backward ops (hand-derived, not autodiff), the ownership of
32x32 dW blocks by waves, the thin-accumulator numbering, and an LDS slot plan.

Row-locality: GlobalAveragePooling2D / Reshape / Flatten / Lambda are identities per row only when
the feature map is 1x1 (P == 1), which is how the reference trains and evaluates
(train_96.py:134-140, test.py:31).  For P > 1 such graphs raise ValueError (the SE/MHA spatial
stages are a separate kernel path).
"""
import math
import os
import struct

import numpy as np

# ---- word layout (mirror of csrc/hpe_prog.h) -----------------------------------------------------
HPE_MAGIC = 0x31455048
(H_MAGIC, H_NOPS, H_NSLOTS, H_T, H_NW, H_IN_SLOT, H_OUT_SLOT, H_CIN, H_COUT, H_NPARAMS,
 H_NPARAMS_TRAIN, H_LDS_FLOATS, H_MAXACC, H_MAXTHIN, H_NTACC, H_OPS_OFF, H_SLOTS_OFF, H_BLK_OFF,
 H_TACC_OFF, H_MODE, H_WG_PER_CU, H_SCRATCH_OFF, H_NTHIN, H_SLAB, H_KIND, H_NPASS, H_GSLOTS) = range(27)
H_WORDS = 32
MODE_FWD, MODE_TRAIN, MODE_EVAL = 0, 1, 2
S_WORDS = 4
(O_TYPE, O_A, O_B, O_OUT, O_K, O_N, O_W, O_BIAS, O_FLAGS, O_EACT, O_EDROP, O_ETHR, O_EKEEP, O_EZ,
 O_AUX0, O_AUX1, O_AUX2, O_AUX3, O_TBASE, O_TCOUNT, O_F0, O_F1, O_MODE, O_WSEL) = range(24)
O_WORDS = 24
(OP_DENSE, OP_TDENSE, OP_EW, OP_LN, OP_LOSS, OP_EPIGRAD, OP_DW, OP_TACC, OP_DIN, OP_TDIN, OP_EWB,
 OP_LNB, OP_MLP2, OP_CHAIN, OP_RES) = range(1, 16)
RL_WORDS = 8           # residual-stack layer table entry (csrc/hpe_prog.h RL_*)
EW_HAS_B, EW_MUL, EW_AFFINE = 1, 2, 4
DST_STORE, DST_ACCUM, DST_EPIGRAD = 0, 1, 2
TACC_GEMM, TACC_BIAS, TACC_DIAG = 0, 1, 2
ACTS = {None: 0, 'linear': 0, 'tanh': 1, 'relu': 2, 'softsign': 3, 'sigmoid': 4, 'elu': 5,
        'selu': 6, 'swish': 7, 'softplus': 8, 'leaky_relu': 9}
NEEDS_Z = {7}          # swish: derivative needs the pre-activation
THIN_N = 8             # N <= THIN_N -> VALU path
MAXTHIN = 4
ACC_VARIANTS = (1, 2, 4, 8)
NW_VARIANTS = (4, 8, 12, 16)
LDS_LIMIT_FLOATS = 160 * 1024 // 4 - 32
FWD_NW = int(os.environ.get('HPE_FWD_NW', '8'))   # waves of generic inference programs (16 spills)
GS_NW = 16             # global-slot programs (slot plan > LDS) run the 16-wave kernel
GS_T = 32


def _f2i(x):
    return struct.unpack('<i', struct.pack('<f', float(x)))[0]


def _u2i(x):
    x = int(x) & 0xFFFFFFFF
    return x - (1 << 32) if x >= (1 << 31) else x


def act_id(name):
    if name not in ACTS:
        raise ValueError('Unknown activation function: %r' % (name,))
    return ACTS[name]


def slot_geometry(C):
    """Padded channel count (multiple of 8, so Kh = Cp/2 is a multiple of 4) and a row stride of
    4*odd floats: ds_read_b128 by 16 consecutive rows hits 16 distinct bank quads."""
    cp = max(8, -(-C // 8) * 8)
    st = cp if (cp // 4) % 2 == 1 else cp + 4
    return cp, st


def dropout_threshold(rate):
    return min(int(math.floor(float(rate) * 4294967296.0)), 4294967295)


# ==================================================================================================
# intermediate representation
# ==================================================================================================
class Tensor:
    def __init__(self, tid, C, name):
        self.id, self.C, self.name = tid, C, name
        self.producer = None     # FOp
        self.consumers = []      # FOp list (with multiplicity)
        self.slot = None         # value slot
        self.gslot = None        # gradient slot (may == slot when in place)
        self.gstate = 0          # 0 none, 1 stored (partial), 2 final-pre-epilogue


class FOp:
    """Forward op.  kind: dense | ew | ln."""

    def __init__(self, kind, ins, out, **kw):
        self.kind, self.ins, self.out = kind, ins, out
        self.act, self.drop_id, self.rate = 0, -1, 0.0
        self.zt = None           # tensor holding pre-activation (swish)
        self.__dict__.update(kw)

    def epi_trivial(self):
        return self.act == 0 and self.drop_id < 0


class Program:
    """Result of compile_graph: words + parameter layout metadata."""

    def __init__(self):
        self.words = None
        self.n_params = 0
        self.n_train = 0
        self.param_index = {}    # weight key -> (offset, shape)
        self.consts = None       # np.float32 array appended after trainable params
        self.l2 = None           # per-param L2 coefficient (trainable part)
        self.tpos = None         # per-param index into the transposed mirror (-1 none)
        self.n_mirror = 0
        self.mirror_src = []     # (param_off, K, N, mirror_off)
        self.T = 64
        self.NW = 8
        self.mode = MODE_FWD
        self.C_in = 0
        self.C_out = 3
        self.info = {}


# ==================================================================================================
# graph flattening (nested Functional -> prefixed layers)
# ==================================================================================================
def _inbound(l):
    if not l.get('inbound_nodes'):
        return [], {}
    node = l['inbound_nodes'][0]
    ins = [t[0] for t in node]
    kw = {}
    for t in node:
        for k, ref in (t[3] if len(t) > 3 else {}).items():
            if isinstance(ref, list) and ref and isinstance(ref[0], str):
                kw[k] = ref[0]
    return ins, kw


def flatten_layers(model_config, prefix=''):
    """Return (layers in evaluation order, input name, output names); nested models inlined."""
    mc = model_config.get('config', model_config)
    out = []
    alias = {}
    for l in mc['layers']:
        name = prefix + l['name']
        ins, kw = _inbound(l)
        ins = [alias.get(prefix + i, prefix + i) for i in ins]
        kw = {k: alias.get(prefix + v, prefix + v) for k, v in kw.items()}
        if l['class_name'] == 'Functional':
            sub, sin, souts = flatten_layers(l['config'], prefix + l['name'] + '/')
            # the nested input layer aliases this call's input
            for s in sub:
                if s['name'] == sin:
                    s = dict(s, class_name='Identity', ins=ins, kw={})
                out.append(s)
            alias[name] = souts[0]
            continue
        out.append({'name': name, 'class_name': l['class_name'], 'config': l['config'],
                    'ins': ins, 'kw': kw, 'prefix': prefix})
    inp = prefix + mc['input_layers'][0][0]
    outs = [alias.get(prefix + t[0], prefix + t[0]) for t in mc['output_layers']]
    return out, inp, outs


def _topo(layers, outs):
    by = {l['name']: l for l in layers}
    seen, order = set(), []

    def visit(n):
        if n in seen:
            return
        seen.add(n)
        l = by[n]
        for i in l['ins'] + list(l['kw'].values()):
            visit(i)
        order.append(l)
    for o in outs:
        visit(o)
    return order


# ==================================================================================================
# compiler
# ==================================================================================================
class _Builder:
    def __init__(self, weights, mode, P, train_keys):
        self.w = weights
        self.mode = mode
        self.P = P
        self.tensors = []
        self.fops = []
        self.params = []         # list of (key, array) trainable, Keras order
        self.pidx = {}
        self.consts = []         # list of arrays
        self.const_off = 0
        self.l2 = {}
        self.drop_count = 0
        self.train_keys = train_keys

    # -- tensors / params ---------------------------------------------------------------------
    def tensor(self, C, name):
        t = Tensor(len(self.tensors), C, name)
        self.tensors.append(t)
        return t

    def param(self, key):
        if key not in self.pidx:
            raise ValueError('missing weight %r' % key)
        return self.pidx[key][0]

    def const(self, arr):
        arr = np.asarray(arr, dtype=np.float32).ravel()
        off = self.const_off
        self.consts.append(arr)
        self.const_off += arr.size
        return ('const', off)

    # -- epilogue fusion (peephole over the finished forward op list) ----------------------------
    def fuse_epilogues(self):
        """Fold a unary copy op carrying only (activation, dropout) into its producer's epilogue
        when the producer's output has no other consumer: drop_e(act_e(act_p(z))) with at most one
        non-linear activation and the producer not yet dropping."""
        changed = True
        while changed:
            changed = False
            for e in list(self.fops):
                if e.kind != 'ew' or e.flags != 0 or e.f0 != 1.0:
                    continue
                t = e.ins[0]
                p = t.producer
                if p is None or len(t.consumers) != 1 or p.drop_id >= 0:
                    continue
                if p.act != 0 and e.act != 0:
                    continue
                if e.act != 0:
                    p.act = e.act
                if e.drop_id >= 0:
                    p.drop_id, p.rate = e.drop_id, e.rate
                p.out = e.out
                e.out.producer = p
                t.producer = None
                t.consumers = []
                self.fops.remove(e)
                changed = True

    def add(self, fop):
        for t in fop.ins:
            t.consumers.append(fop)
        fop.out.producer = fop
        self.fops.append(fop)
        return fop.out


def _reg(cfg, key):
    r = cfg.get(key)
    if not r:
        return 0.0
    if r.get('class_name') in ('L2', 'L1L2'):
        return float(np.float32(r.get('config', {}).get('l2', 0.0)))
    return 0.0


def compile_graph(model_config, weights, mode='fwd', P=1, T=None, NW=None, wg_per_cu=0,
                  trainable=None, fused=True, rbw=1):
    """Compile to a Program.  weights: dict key -> np.ndarray (Keras '<layer>/<var>' keys)."""
    modes = {'fwd': MODE_FWD, 'train': MODE_TRAIN, 'eval': MODE_EVAL}
    if mode not in modes:
        raise ValueError('mode must be fwd|train|eval')
    training = mode == 'train'
    layers, inp, outs = flatten_layers(model_config)
    if len(outs) != 1:
        raise ValueError('row programs need a single-output graph (got %d outputs)' % len(outs))
    order = _topo(layers, outs)
    b = _Builder(weights, mode, P, trainable)
    b.drop_ids = {l['name']: i for i, l in enumerate(
        [l for l in layers if l['class_name'] in ('SpatialDropout2D', 'Dropout')])}

    # parameter layout: trainable weights in Keras trainable_weights order (layer order, kernel
    # before bias; MHA query/key/value/output) -- the same flat order the optimizer state uses.
    rank = {'kernel': 0, 'depthwise_kernel': 0, 'pointwise_kernel': 1, 'bias': 2, 'gamma': 0,
            'beta': 1}
    subrank = {'query': 0, 'key': 1, 'value': 2, 'attention_output': 3}
    off = 0
    l2c = []
    for l in layers:
        pre = l['name'] + '/'
        keys = [k for k in weights if k.startswith(pre) and '/' not in k[len(pre):].replace(
            'query/', '').replace('key/', '').replace('value/', '').replace('attention_output/', '')]
        keys = [k for k in keys if k.rsplit('/', 1)[-1] in rank]

        def kk(k):
            parts = k[len(pre):].split('/')
            return (subrank.get(parts[0], 0) if len(parts) > 1 else 0, rank[parts[-1]])
        for k in sorted(keys, key=kk):
            a = np.asarray(weights[k], dtype=np.float32)
            b.params.append((k, a))
            b.pidx[k] = (off, a.shape)
            base = k.rsplit('/', 1)[-1]
            cfg = l['config']
            if base in ('kernel', 'depthwise_kernel', 'pointwise_kernel'):
                c2 = _reg(cfg, 'kernel_regularizer')
                if base == 'depthwise_kernel':
                    c2 = _reg(cfg, 'depthwise_regularizer') or c2
                if base == 'pointwise_kernel':
                    c2 = _reg(cfg, 'pointwise_regularizer') or c2
            elif base == 'bias' and l['class_name'] != 'MultiHeadAttention':
                c2 = _reg(cfg, 'bias_regularizer')
            else:
                c2 = 0.0
            l2c.append(np.full(a.size, c2, dtype=np.float32))
            off += a.size
    n_train = off

    # transposed mirror of every 2-D weight block a GEMM can read (fixed per model, any mode)
    b.mirror = []
    mo = 0
    for l in layers:
        cls = l['class_name']
        blocks = []
        try:
            if cls in ('Conv2D', 'Dense', 'Conv2DTranspose'):
                b.P, saved = 1, b.P
                w, K, N, _, tr = _dense_params(b, l)
                b.P = saved
                blocks.append((w[1], N, K) if tr else (w[1], K, N))
            elif cls == 'SeparableConv2D':
                pk = l['name'] + '/pointwise_kernel'
                _, _, C2, N = b.pidx[pk][1]
                blocks.append((b.param(pk), C2, N))
            elif cls == 'MultiHeadAttention':
                for part in ('value', 'attention_output'):
                    key = l['name'] + '/' + part + '/kernel'
                    shp = b.pidx[key][1]
                    K = int(np.prod(shp[:-1])) if part == 'attention_output' else shp[0]
                    N = int(np.prod(shp)) // K
                    blocks.append((b.param(key), K, N))
        except ValueError:
            b.P = P
            blocks = []
        for (o, K, N) in blocks:
            b.mirror.append((o, K, N, mo))
            mo += K * N

    # ---- forward lowering --------------------------------------------------------------------
    tmap = {}
    cin = None
    for l in order:
        if l['name'] == inp or l['class_name'] == 'InputLayer' and not l['ins']:
            cfg = l['config']
            cin = cfg['batch_input_shape'][-1]
            t = b.tensor(cin, l['name'])
            tmap[l['name']] = t
            continue
        _lower(b, l, tmap, training, P)
    x_t = tmap[inp]
    y_t = tmap[outs[0]]
    if y_t is x_t:
        raise ValueError('model output is its input')
    b.fuse_epilogues()
    live = {x_t.id} | {f.out.id for f in b.fops}
    b.tensors = [t for t in b.tensors if t.id in live]
    if fused:
        if mode == 'fwd':
            ch = _try_chain(b, x_t, y_t, n_train, l2c)
            if ch is not None:
                return ch
        mlp2 = _try_mlp2(b, x_t, y_t, modes[mode], n_train, l2c, P)
        if mlp2 is not None:
            return mlp2
        if mode == 'train':
            res = _try_res(b, x_t, y_t, n_train, l2c)
            if res is not None:
                return res
    prog = _finish(b, x_t, y_t, modes[mode], training, P, T, NW, wg_per_cu, n_train, l2c)
    prog.kind = 'generic'
    return prog


def _dense_params(b, l):
    """(w_ref, K, N, bias_ref, wsel_transposed) for Conv2D/Dense-like layers on 1x1 rows."""
    cls, cfg, name = l['class_name'], l['config'], l['name']
    use_bias = cfg.get('use_bias', True)
    if cls == 'Dense':
        key = name + '/kernel'
        K, N = b.pidx[key][1]
        return ('p', b.param(key)), K, N, ('p', b.param(name + '/bias')) if use_bias else None, False
    if cls == 'Conv2D':
        key = name + '/kernel'
        kh, kw, K, N = b.pidx[key][1]
        if tuple(cfg.get('strides', (1, 1))) != (1, 1) or tuple(cfg.get('dilation_rate', (1, 1))) != (1, 1):
            raise ValueError('Conv2D %s: only stride 1 / dilation 1 on the row path' % name)
        if (kh, kw) != (1, 1):
            if b.P != 1 or cfg.get('padding') != 'same' or kh % 2 == 0 or kw % 2 == 0:
                raise ValueError('Conv2D %s: %dx%d kernel is row-local only on 1x1 maps with '
                                 "'same' padding" % (name, kh, kw))
        centre = ((kh // 2) * kw + kw // 2) * K * N
        return (('p', b.param(key) + centre), K, N,
                ('p', b.param(name + '/bias')) if use_bias else None, False)
    if cls == 'Conv2DTranspose':
        key = name + '/kernel'
        kh, kw, N, K = b.pidx[key][1]
        if b.P != 1 or kh % 2 == 0 or kw % 2 == 0 or tuple(cfg.get('strides', (1, 1))) != (1, 1):
            raise ValueError('Conv2DTranspose %s: row-local only on 1x1 maps, stride 1' % name)
        centre = ((kh // 2) * kw + kw // 2) * K * N
        # centre tap is stored [out][in] = W^T: read it through the mirror buffer
        return (('p', b.param(key) + centre), K, N,
                ('p', b.param(name + '/bias')) if use_bias else None, True)
    raise ValueError(cls)


def _emit_dense(b, l, x, w_ref, K, N, bias_ref, transposed, act, name):
    if x.C != K:
        raise ValueError('%s: input has %d channels, kernel expects %d' % (name, x.C, K))
    y = b.tensor(N, name)
    op = FOp('dense', [x], y, K=K, N=N, w=w_ref, bias=bias_ref, transposed=transposed,
             act=act, name=name)
    return b.add(op)


def _lower(b, l, tmap, training, P):
    cls, cfg, name = l['class_name'], l['config'], l['name']
    ins = [tmap[i] for i in l['ins']]
    x = ins[0] if ins else None
    alias_ok = P == 1

    def alias():
        tmap[name] = x

    if cls in ('Identity', 'InputLayer'):
        return alias()
    if cls in ('Conv2D', 'Dense', 'Conv2DTranspose'):
        w, K, N, bias, tr = _dense_params(b, l)
        tmap[name] = _emit_dense(b, l, x, w, K, N, bias, tr, act_id(cfg.get('activation')), name)
        return
    if cls == 'SeparableConv2D':
        dk = name + '/depthwise_kernel'
        kh, kw, C, mult = b.pidx[dk][1]
        if (kh, kw) != (1, 1) or mult != 1:
            raise ValueError('SeparableConv2D %s: only 1x1 depthwise, depth_multiplier 1' % name)
        t = b.tensor(C, name + '/dw')
        b.add(FOp('ew', [x], t, flags=EW_AFFINE, f0=1.0, f1=0.0, scale=('p', b.param(dk)),
                  shift=None, scale_trainable=True, name=name + '/dw'))
        pk = name + '/pointwise_kernel'
        _, _, C2, N = b.pidx[pk][1]
        bias = ('p', b.param(name + '/bias')) if cfg.get('use_bias', True) else None
        tmap[name] = _emit_dense(b, l, t, ('p', b.param(pk)), C2, N, bias, False,
                                 act_id(cfg.get('activation')), name)
        return
    if cls in ('Activation', 'ReLU'):
        if cls == 'ReLU':
            if cfg.get('max_value') is not None or cfg.get('negative_slope', 0) or cfg.get('threshold', 0):
                raise ValueError('ReLU %s: only plain relu supported' % name)
            a = ACTS['relu']
        else:
            a = act_id(cfg['activation'])
        if a == 0:
            return alias()
        t = b.tensor(x.C, name)
        tmap[name] = b.add(FOp('ew', [x], t, flags=0, f0=1.0, f1=0.0, act=a, name=name))
        return
    if cls in ('SpatialDropout2D', 'Dropout'):
        rate = float(cfg['rate'])
        if not 0.0 <= rate <= 1.0:
            raise ValueError('Invalid value %s received for `rate`, expected a value between 0 '
                             'and 1.' % rate)
        did = b.drop_ids[name]   # ordinal in model_config layer order (oracle numbering)
        if not training or rate == 0.0:
            return alias()
        t = b.tensor(x.C, name)
        tmap[name] = b.add(FOp('ew', [x], t, flags=0, f0=1.0, f1=0.0, drop_id=did, rate=rate, name=name))
        return
    if cls in ('Add', 'Average'):
        if len({t.C for t in ins}) != 1:
            raise ValueError('%s %s: inputs have different channel counts' % (cls, name))
        if cls == 'Average' and len(ins) != 2:
            raise ValueError('Average with %d inputs not supported' % len(ins))
        f = 0.5 if cls == 'Average' else 1.0
        y = ins[0]
        for i, t in enumerate(ins[1:]):
            o = b.tensor(t.C, name if i == len(ins) - 2 else name + '/%d' % i)
            y = b.add(FOp('ew', [y, t], o, flags=EW_HAS_B, f0=f, f1=f, name=name))
        tmap[name] = y
        return
    if cls == 'Multiply':
        if len(ins) != 2 or ins[0].C != ins[1].C:
            raise ValueError('Multiply %s: two inputs with equal channels required' % name)
        if not alias_ok:
            raise ValueError('Multiply with a per-image gate needs P == 1 on the row path')
        o = b.tensor(ins[0].C, name)
        tmap[name] = b.add(FOp('ew', ins, o, flags=EW_HAS_B | EW_MUL, f0=1.0, f1=1.0, name=name))
        return
    if cls in ('Flatten', 'Reshape', 'Lambda', 'GlobalAveragePooling2D'):
        if not alias_ok:
            raise ValueError('%s %s is row-local only on 1x1 feature maps (P == 1)' % (cls, name))
        if cls == 'Lambda' and len(ins) == 2:
            tmap[name] = ins[0]   # reshape_back(t, orig): per row, t itself
            return
        return alias()
    if cls == 'BatchNormalization':
        if training:
            raise ValueError('BatchNormalization training mode is not on the hot path')
        eps = float(cfg['epsilon'])
        mean = b.w[name + '/moving_mean'].astype(np.float64)
        var = b.w[name + '/moving_variance'].astype(np.float64)
        g = b.w[name + '/gamma'].astype(np.float64) if cfg.get('scale', True) else 1.0
        be = b.w[name + '/beta'].astype(np.float64) if cfg.get('center', True) else 0.0
        s = np.float32(1.0) / np.sqrt(np.float32(var) + np.float32(eps))
        s = (s * np.float32(g)).astype(np.float32)
        sh = (np.float32(be) - np.float32(mean) * s).astype(np.float32)
        o = b.tensor(x.C, name)
        tmap[name] = b.add(FOp('ew', [x], o, flags=EW_AFFINE, f0=1.0, f1=0.0, scale=b.const(s),
                               shift=b.const(sh), scale_trainable=False, name=name))
        return
    if cls == 'LayerNormalization':
        ax = cfg.get('axis')
        if isinstance(ax, list) and len(ax) != 1:
            raise ValueError('LayerNormalization over several axes not supported')
        o = b.tensor(x.C, name)
        g = ('p', b.param(name + '/gamma')) if cfg.get('scale', True) else None
        be = ('p', b.param(name + '/beta')) if cfg.get('center', True) else None
        tmap[name] = b.add(FOp('ln', [x], o, gamma=g, beta=be, eps=float(cfg['epsilon']), name=name))
        return
    if cls == 'MultiHeadAttention':
        if not alias_ok:
            raise ValueError('MultiHeadAttention over H*W > 1 tokens is not row-local (P must be 1)')
        # one token: softmax == 1, output = (value(x) . Wo + bo) -- attention_model.py:52-55
        v_in = tmap[l['kw']['value']] if 'value' in l['kw'] else (ins[1] if len(ins) > 1 else x)
        vk = name + '/value/kernel'
        C, h, d = b.pidx[vk][1]
        t = _emit_dense(b, l, v_in, ('p', b.param(vk)), C, h * d,
                        ('p', b.param(name + '/value/bias')) if cfg.get('use_bias', True) else None,
                        False, 0, name + '/value')
        ok = name + '/attention_output/kernel'
        h2, d2, Co = b.pidx[ok][1]
        tmap[name] = _emit_dense(b, l, t, ('p', b.param(ok)), h2 * d2, Co,
                                 ('p', b.param(name + '/attention_output/bias')) if cfg.get('use_bias', True) else None,
                                 False, 0, name)
        return
    raise ValueError('layer %s (%s) is not supported on the row path' % (name, cls))


# ==================================================================================================
# backward construction + emission
# ==================================================================================================
class _Emit:
    def __init__(self):
        self.ops = []            # list of dicts (word fields)
        self.slots = []          # [C]
        self.slot_names = []

    def slot(self, C, name=''):
        self.slots.append(C)
        self.slot_names.append(name)
        return len(self.slots) - 1

    def op(self, f):
        d = {k: 0 for k in range(O_WORDS)}
        for k in (O_A, O_B, O_OUT, O_BIAS, O_EDROP, O_EZ, O_AUX0, O_AUX1, O_AUX2, O_AUX3):
            d[k] = -1
        d[O_EKEEP] = _f2i(1.0)
        d.update(f)
        self.ops.append(d)
        return len(self.ops) - 1


def _epi_fields(op, zslot=-1):
    if op is None:
        return {}
    d = {O_EACT: op.act, O_EZ: zslot}
    if op.drop_id >= 0:
        d[O_EDROP] = op.drop_id
        d[O_ETHR] = _u2i(dropout_threshold(op.rate))
        d[O_EKEEP] = _f2i(np.float32(1.0) - np.float32(op.rate))
    return d


def _finish(b, x_t, y_t, mode, training, P, T, NW, wg_per_cu, n_train, l2c):
    E = _Emit()
    # value slots
    for t in b.tensors:
        t.slot = E.slot(t.C, t.name)
    # pre-activation slots (swish)
    for f in b.fops:
        if f.act in NEEDS_Z and training:
            f.zt = E.slot(f.out.C, f.out.name + '/z')

    # parameter reference resolution: ('p', off) -> params word offset; ('const', off) -> after
    def ref(r):
        if r is None:
            return -1
        return r[1] if r[0] == 'p' else n_train + r[1]

    mirror = b.mirror        # model-level: (param_off, rows, cols, mirror_off), mode-independent

    def mirror_of(w_off, K, N):
        for (o, k, n, mo) in mirror:
            if o == w_off and k == K and n == N:
                return mo
        raise ValueError('no transposed mirror for weight block at %d (%dx%d)' % (w_off, K, N))

    fwd_idx = {}
    for f in b.fops:
        zslot = f.zt if f.zt is not None else -1
        if f.kind == 'dense':
            thin = f.N <= THIN_N
            w_off = ref(f.w)
            wsel = 0
            if f.transposed:
                # weights stored [N][K] -> the [K][N] layout lives in the mirror
                wsel = 1
                w_off = mirror_of(w_off, f.N, f.K)
            fields = {O_TYPE: OP_TDENSE if thin else OP_DENSE, O_A: f.ins[0].slot, O_OUT: f.out.slot,
                      O_K: f.K, O_N: f.N, O_W: w_off, O_BIAS: ref(f.bias), O_WSEL: wsel}
            if thin:
                fields[O_AUX3] = 0   # ksplit filled below
            fields.update(_epi_fields(f, zslot))
            fwd_idx[f] = E.op(fields)
        elif f.kind == 'ew':
            fields = {O_TYPE: OP_EW, O_A: f.ins[0].slot, O_OUT: f.out.slot, O_FLAGS: f.flags,
                      O_F0: _f2i(f.f0), O_F1: _f2i(f.f1)}
            if f.flags & EW_HAS_B:
                fields[O_B] = f.ins[1].slot
            if f.flags & EW_AFFINE:
                fields[O_AUX0] = ref(f.scale)
                fields[O_AUX1] = ref(f.shift)
            fields.update(_epi_fields(f, zslot))
            fwd_idx[f] = E.op(fields)
        elif f.kind == 'ln':
            f.xhat = E.slot(f.out.C, f.out.name + '/xhat') if training else -1
            f.rstd = E.slot(1, f.out.name + '/rstd') if training else -1
            fields = {O_TYPE: OP_LN, O_A: f.ins[0].slot, O_OUT: f.out.slot,
                      O_AUX0: ref(f.gamma), O_AUX1: ref(f.beta), O_AUX2: f.xhat, O_AUX3: f.rstd,
                      O_F0: _f2i(f.eps)}
            fields.update(_epi_fields(f, zslot))
            fwd_idx[f] = E.op(fields)

    dw_blocks = []           # (op index, kb, nb)
    tacc_ops = []
    nthin = 0

    def tacc(a_slot, b_slot, K, N, tmode, poff):
        nonlocal nthin
        cnt = K * N if tmode == TACC_GEMM else N
        i = E.op({O_TYPE: OP_TACC, O_A: a_slot, O_B: b_slot, O_K: K, O_N: N, O_AUX3: tmode,
                    O_TBASE: nthin, O_TCOUNT: cnt, O_W: poff})
        tacc_ops.append(i)
        nthin += cnt

    if mode != MODE_FWD:
        y_prod = y_t.producer
        E.op({O_TYPE: OP_LOSS, O_A: y_t.slot, O_OUT: y_t.slot, O_N: y_t.C,
                **_epi_fields(y_prod, y_prod.zt if (y_prod and y_prod.zt is not None) else -1)})
    if training:
        y_t.gslot = y_t.slot
        y_t.gstate = 2       # gradient wrt y's producer pre-epilogue, in place
        pending = {}         # tensor -> number of consumers whose backward is still to run
        for t in b.tensors:
            pending[t.id] = len(t.consumers)

        def ensure_pre_epi(t):
            """Make t.gslot hold the gradient wrt t's producer pre-epilogue output."""
            p = t.producer
            if t.gstate == 2 or p is None:
                return
            if p.epi_trivial():
                t.gstate = 2
                return
            E.op({O_TYPE: OP_EPIGRAD, O_A: t.slot, O_OUT: t.gslot,
                    **_epi_fields(p, p.zt if p.zt is not None else -1)})
            t.gstate = 2

        def grad_dest(t):
            """Destination (slot, mode, epi-producer) for a gradient written into tensor t."""
            if t is x_t:
                return None
            single = len(t.consumers) == 1
            if single:
                t.gslot = t.slot
                p = t.producer
                if p is not None and not p.epi_trivial():
                    t.gstate = 2
                    return (t.slot, DST_EPIGRAD, p)
                t.gstate = 2
                return (t.slot, DST_STORE, None)
            if t.gslot is None:
                t.gslot = E.slot(t.C, t.name + '/grad')
                t.gstate = 1
                return (t.gslot, DST_STORE, None)
            return (t.gslot, DST_ACCUM, None)

        for f in reversed(b.fops):
            t = f.out
            if t.gslot is None:
                continue     # no gradient reaches this op (e.g. unused branch)
            ensure_pre_epi(t)
            g = t.gslot
            if f.kind == 'dense':
                x = f.ins[0]
                thin = f.N <= THIN_N
                w_off = ref(f.w)
                if f.transposed:
                    raise ValueError('%s: Conv2DTranspose training is not on the hot path' % f.name)
                if thin:
                    tacc(x.slot, g, f.K, f.N, TACC_GEMM, w_off)
                else:
                    iop = E.op({O_TYPE: OP_DW, O_A: x.slot, O_B: g, O_K: f.K, O_N: f.N, O_W: w_off})
                    for kb in range(-(-f.K // 32)):
                        for nb in range(-(-f.N // 32)):
                            dw_blocks.append((iop, kb, nb))
                if f.bias is not None:
                    tacc(-1, g, 1, f.N, TACC_BIAS, ref(f.bias))
                dst = grad_dest(x)
                if dst is not None:
                    dslot, dmode, prod = dst
                    fields = {O_A: g, O_OUT: dslot, O_K: f.K, O_N: f.N, O_MODE: dmode,
                              O_AUX0: x.slot}
                    if f.N <= THIN_N:   # TDIN reads W [K][N] in place
                        fields.update({O_TYPE: OP_TDIN, O_W: ref(f.w), O_WSEL: 0})
                    else:               # DIN reads the mirror W^T [N][K] (params_t)
                        fields.update({O_TYPE: OP_DIN, O_W: mirror_of(ref(f.w), f.K, f.N), O_WSEL: 0})
                    if prod is not None:
                        fields.update(_epi_fields(prod, prod.zt if prod.zt is not None else -1))
                    E.op(fields)
            elif f.kind == 'ew':
                if f.flags & EW_AFFINE and getattr(f, 'scale_trainable', False):
                    tacc(f.ins[0].slot, g, f.ins[0].C, f.ins[0].C, TACC_DIAG, ref(f.scale))
                dsts = []
                for i, xin in enumerate(f.ins):
                    d = grad_dest_plain(xin, E, x_t)
                    dsts.append(d)
                fields = {O_TYPE: OP_EWB, O_A: f.ins[0].slot, O_OUT: g, O_FLAGS: f.flags,
                          O_F0: _f2i(f.f0), O_F1: _f2i(f.f1), O_AUX2: ref(getattr(f, 'scale', None))}
                if f.flags & EW_HAS_B:
                    fields[O_B] = f.ins[1].slot
                m = 0
                if dsts[0] is not None:
                    fields[O_AUX0] = dsts[0][0]
                    m |= 1 if dsts[0][1] == DST_ACCUM else 0
                if len(dsts) > 1 and dsts[1] is not None:
                    fields[O_AUX1] = dsts[1][0]
                    m |= 2 if dsts[1][1] == DST_ACCUM else 0
                fields[O_MODE] = m
                E.op(fields)
            elif f.kind == 'ln':
                if f.gamma is not None:
                    tacc(f.xhat, g, f.out.C, f.out.C, TACC_DIAG, ref(f.gamma))
                if f.beta is not None:
                    tacc(-1, g, 1, f.out.C, TACC_BIAS, ref(f.beta))
                d = grad_dest_plain(f.ins[0], E, x_t)
                if d is not None:
                    E.op({O_TYPE: OP_LNB, O_A: f.xhat, O_B: g, O_OUT: d[0],
                            O_AUX0: ref(f.gamma), O_AUX1: f.rstd, O_MODE: d[1]})

    # ---- geometry: T / NW / thin split / slot plan ---------------------------------------------
    ndw = len(dw_blocks)
    cand_nw = [NW] if NW else list(NW_VARIANTS)
    best = None
    for nw in cand_nw:
        nt = nw * 64
        if training and -(-nthin // nt) > MAXTHIN:
            continue
        macc = -(-ndw // nw) if ndw else 1
        acc = next((a for a in ACC_VARIANTS if a >= macc), None)
        if acc is None:
            continue
        # MFMA work balance over waves (forward tasks + dW blocks), prefer fewer idle waves
        score = (acc * nw - ndw if ndw else 0, -nw)
        if best is None or score < best[0]:
            best = (score, nw, acc)
    npass = 1
    if best is None:
        # more dW blocks than one launch's register accumulators: H_NPASS launches per step, each
        # recomputing the tile's forward / backward and owning NW * 8 blocks
        nw = max(cand_nw)
        if -(-nthin // (nw * 64)) > MAXTHIN or nw != max(NW_VARIANTS):
            raise ValueError('model too large for the row kernel: %d dW blocks, %d thin elements'
                             % (ndw, nthin))
        acc = ACC_VARIANTS[-1]
        npass = -(-ndw // (nw * acc))
        best = (None, nw, acc)
    _, nw, acc = best
    if NW is None and not training:
        # inference programs: one workgroup per CU is typical (slot plans of 60-150 KiB), so its
        # waves are the CU's only latency hiding for the per-lane weight loads of OP_DENSE
        nw, acc = FWD_NW, 1
    nt = nw * 64
    # slot layout: live intervals over the op list, first-fit in LDS (every writer re-zeroes a
    # slot's padding columns, so regions can be shared by slots that are never live together)
    live = _liveness(E, x_t.slot, y_t.slot, mode)
    nslots = len(E.slots)

    def plan(Tv):
        sizes = []
        for C in E.slots:
            cp, st = slot_geometry(C)
            sizes.append((C, cp, st, Tv * st))
        items = [(live[i][0], live[i][1], sizes[i][3], i) for i in range(nslots)]
        for j, d in enumerate(E.ops):   # TDENSE scratch: transient pseudo-slot
            if d[O_TYPE] == OP_TDENSE:
                need = Tv * d[O_N] * max(1, min(nt // (Tv * d[O_N]), -(-d[O_K] // 8)))
                items.append((j, j, -(-need // 4) * 4, nslots + j))
        placed = []
        offmap = {}
        for (a0, a1, sz, key) in sorted(items, key=lambda t: (t[0], -t[2])):
            cands = sorted({0} | {p[2] + p[3] for p in placed})
            for o in cands:
                if all(not (a0 <= p1 and p0 <= a1 and o < po + ps and po < o + sz)
                       for (p0, p1, po, ps) in placed):
                    break
            placed.append((a0, a1, o, sz))
            offmap[key] = o
        offs = [(offmap[i],) + sizes[i][:3] for i in range(nslots)]
        scratch_offs = {k - nslots: v for k, v in offmap.items() if k >= nslots}
        top = max([p[2] + p[3] for p in placed] + [0])
        return offs, scratch_offs, top
    cands = [T] if T else [128, 64, 32]
    chosen = None
    gslots = 0
    for Tv in cands:
        offs, scratch, tot = plan(Tv)
        if tot <= LDS_LIMIT_FLOATS:
            chosen = (Tv, offs, scratch, tot)
            break
    if chosen is None:
        # the slot plan does not fit 160 KiB even at the smallest tile: keep the slots in a
        # per-workgroup device scratch region (H_GSLOTS; same interpreter, L2/MALL-resident)
        if NW is not None and NW != GS_NW:
            raise ValueError('row program does not fit LDS even at T=%d' % cands[-1])
        gslots = 1
        if nw != GS_NW:
            nw = GS_NW
            nt = nw * 64
            if ndw:
                acc = next(a for a in ACC_VARIANTS if a >= min(-(-ndw // nw), ACC_VARIANTS[-1]))
                npass = -(-ndw // (nw * acc))
            else:
                acc = 1
        Tv = T or GS_T
        offs, scratch, tot = plan(Tv)
        chosen = (Tv, offs, scratch, tot)
    Tv, offs, scratch_offs, tot = chosen
    for j, d in enumerate(E.ops):
        if d[O_TYPE] == OP_TDENSE:
            d[O_AUX3] = max(1, min(nt // (Tv * d[O_N]), -(-d[O_K] // 8)))
            d[O_AUX2] = scratch_offs[j]
    scratch = 0

    # ---- words --------------------------------------------------------------------------------
    hdr = [0] * H_WORDS
    slots_w = []
    for (o, C, cp, st) in offs:
        slots_w += [o, C, cp, st]
    ops_w = []
    for d in E.ops:
        ops_w += [int(d[k]) for k in range(O_WORDS)]
    blk = [-1] * (npass * nw * acc)
    for j, (iop, kb, nb) in enumerate(dw_blocks):
        pa, jj = divmod(j, nw * acc)
        w_, s_ = jj % nw, jj // nw
        blk[(pa * nw + w_) * acc + s_] = (iop << 16) | (kb << 8) | nb
    n_params = n_train + b.const_off
    hdr[H_MAGIC] = HPE_MAGIC
    hdr[H_NOPS] = len(E.ops)
    hdr[H_NSLOTS] = len(E.slots)
    hdr[H_T] = Tv
    hdr[H_NW] = nw
    hdr[H_IN_SLOT] = x_t.slot
    hdr[H_OUT_SLOT] = y_t.slot
    hdr[H_CIN] = x_t.C
    hdr[H_COUT] = y_t.C
    hdr[H_NPARAMS] = n_params
    hdr[H_NPARAMS_TRAIN] = n_train
    hdr[H_LDS_FLOATS] = -(-tot // 4) * 4
    hdr[H_MAXACC] = acc
    hdr[H_MAXTHIN] = max(1, -(-nthin // nt)) if nthin else 1
    hdr[H_NTACC] = len(tacc_ops)
    hdr[H_SLOTS_OFF] = H_WORDS
    hdr[H_OPS_OFF] = H_WORDS + len(slots_w)
    hdr[H_BLK_OFF] = hdr[H_OPS_OFF] + len(ops_w)
    hdr[H_TACC_OFF] = hdr[H_BLK_OFF] + len(blk)
    hdr[H_MODE] = mode
    hdr[H_WG_PER_CU] = wg_per_cu
    hdr[H_SCRATCH_OFF] = scratch
    hdr[H_NTHIN] = nthin
    hdr[H_SLAB] = -(-(n_train + 4) // 4) * 4
    hdr[H_NPASS] = npass
    hdr[H_GSLOTS] = gslots
    words = np.asarray(hdr + slots_w + ops_w + blk + tacc_ops, dtype=np.int64)
    words = ((words + (1 << 31)) % (1 << 32) - (1 << 31)).astype(np.int32)

    prog = Program()
    prog.words = words
    prog.n_params = n_params
    prog.n_train = n_train
    prog.param_index = {k: b.pidx[k] for k, _ in b.params}
    prog.param_keys = [k for k, _ in b.params]
    prog.consts = np.concatenate(b.consts).astype(np.float32) if b.consts else np.zeros(0, np.float32)
    prog.l2 = np.concatenate(l2c).astype(np.float32) if l2c else np.zeros(0, np.float32)
    prog.n_mirror = sum(k * n for _, k, n, _ in mirror)
    prog.mirror = list(mirror)
    tpos = np.full(n_train, -1, dtype=np.int32)
    for (o, K, N, mo) in mirror:
        if o < n_train:
            idx = np.arange(K * N)
            k_, n_ = idx // N, idx % N
            tpos[o + idx] = mo + n_ * K + k_
    prog.tpos = tpos
    prog.T, prog.NW, prog.mode = Tv, nw, mode
    prog.C_in, prog.C_out = x_t.C, y_t.C
    prog.info = {'ops': len(E.ops), 'slots': len(E.slots), 'dw_blocks': ndw, 'thin': nthin,
                 'maxacc': acc, 'lds_bytes': hdr[H_LDS_FLOATS] * 4, 'npass': npass, 'gslots': gslots}
    return prog


def grad_dest_plain(t, E, x_t):
    """Gradient destination for EWB / LNB (store/accumulate only; epilogue handled separately)."""
    if t is x_t:
        return None
    if len(t.consumers) == 1 and (t.producer is None or t.producer.epi_trivial()):
        t.gslot = t.slot
        t.gstate = 2
        return (t.slot, DST_STORE)
    if t.gslot is None:
        t.gslot = E.slot(t.C, t.name + '/grad')   # value kept for the producer's epilogue grad
        t.gstate = 1
        return (t.gslot, DST_STORE)
    return (t.gslot, DST_ACCUM)


def build_mirror(prog, params):
    """Transposed copies [N][K] of every kernel that a backward GEMM / transposed layer reads."""
    mt = np.zeros(max(prog.n_mirror, 1), dtype=np.float32)
    for (o, K, N, mo) in prog.mirror:
        w = params[o:o + K * N].reshape(K, N)
        mt[mo:mo + K * N] = w.T.ravel()
    return mt


def _liveness(E, in_slot, out_slot, mode):
    """[first def, last use] op index per slot (tile load = -1, output write = len(ops))."""
    n = len(E.slots)
    first = [None] * n
    last = [-1] * n

    def rd(i, s):
        if s is not None and s >= 0:
            last[s] = max(last[s], i)
            if first[s] is None:
                first[s] = i

    def wr(i, s):
        if s is not None and s >= 0:
            if first[s] is None:
                first[s] = i
            last[s] = max(last[s], i)
    wr(-1, in_slot)
    for i, d in enumerate(E.ops):
        t = d[O_TYPE]
        if t in (OP_DENSE, OP_TDENSE):
            rd(i, d[O_A]); wr(i, d[O_OUT]); wr(i, d[O_EZ])
        elif t == OP_EW:
            rd(i, d[O_A])
            if d[O_FLAGS] & EW_HAS_B:
                rd(i, d[O_B])
            wr(i, d[O_OUT]); wr(i, d[O_EZ])
        elif t == OP_LN:
            rd(i, d[O_A]); wr(i, d[O_OUT]); wr(i, d[O_AUX2]); wr(i, d[O_AUX3])
        elif t == OP_LOSS:
            rd(i, d[O_A]); rd(i, d[O_EZ]); wr(i, d[O_OUT])
        elif t == OP_EPIGRAD:
            rd(i, d[O_A]); rd(i, d[O_EZ]); rd(i, d[O_OUT]); wr(i, d[O_OUT])
        elif t in (OP_DW, OP_TACC):
            rd(i, d[O_A]); rd(i, d[O_B])
        elif t in (OP_DIN, OP_TDIN):
            rd(i, d[O_A]); rd(i, d[O_AUX0]); rd(i, d[O_EZ])
            if d[O_MODE] != DST_STORE:
                rd(i, d[O_OUT])
            wr(i, d[O_OUT])
        elif t == OP_EWB:
            rd(i, d[O_OUT]); rd(i, d[O_A])
            if d[O_FLAGS] & EW_HAS_B:
                rd(i, d[O_B])
            wr(i, d[O_AUX0]); wr(i, d[O_AUX1])
            if d[O_MODE] & 1:
                rd(i, d[O_AUX0])
            if d[O_MODE] & 2:
                rd(i, d[O_AUX1])
        elif t == OP_LNB:
            rd(i, d[O_A]); rd(i, d[O_B]); rd(i, d[O_AUX1])
            if d[O_MODE] == DST_ACCUM:
                rd(i, d[O_OUT])
            wr(i, d[O_OUT])
    if mode == MODE_FWD:
        rd(len(E.ops), out_slot)
    return [((first[s] if first[s] is not None else -1), max(last[s], first[s] if first[s] is not None else -1))
            for s in range(n)]


MLP2_MAX_F = 384


def _try_mlp2(b, x_t, y_t, mode, n_train, l2c, P, rbw=1):
    """Recognise the reference's dominant 2-layer regressor (train_96.py:65-110 create_model,
    train_88.py:66-158 / 226-253): x -> dense F (act, dropout) -> dense 3 (act, dropout), and
    emit a KIND_MLP2 program for the fused kernel (csrc/hpe_mlp2.hip)."""
    if len(b.fops) != 2:
        return None
    f1, f2 = b.fops
    if f1.kind != 'dense' or f2.kind != 'dense' or f1.ins[0] is not x_t or f2.ins[0] is not f1.out:
        return None
    if f2.out is not y_t or len(f1.out.consumers) != 1 or f1.transposed or f2.transposed:
        return None
    cin, F, n2 = f1.K, f1.N, f2.N
    if n2 != 3 or cin % 4 or (cin + 7) // 8 * 4 not in (44, 48) or F > MLP2_MAX_F or F < 1:
        return None
    if f1.act in NEEDS_Z or f2.act in NEEDS_Z:
        return None
    if f1.w[0] != 'p' or f2.w[0] != 'p':
        return None

    def ref(r):
        if r is None:
            return -1
        return r[1] if r[0] == 'p' else n_train + r[1]
    ncb = -(-F // 32)
    op = [0] * O_WORDS
    op[O_TYPE] = OP_MLP2
    op[O_K], op[O_N], op[O_AUX3] = cin, F, n2
    op[O_W], op[O_BIAS], op[O_AUX0], op[O_AUX1] = ref(f1.w), ref(f1.bias), ref(f2.w), ref(f2.bias)
    op[O_EACT], op[O_EDROP], op[O_ETHR], op[O_EKEEP], op[O_EZ] = f1.act, -1, 0, _f2i(1.0), -1
    if f1.drop_id >= 0 and mode == MODE_TRAIN:
        op[O_EDROP], op[O_ETHR] = f1.drop_id, _u2i(dropout_threshold(f1.rate))
        op[O_EKEEP] = _f2i(np.float32(1.0) - np.float32(f1.rate))
    op[O_AUX2], op[O_TBASE], op[O_TCOUNT], op[O_F0] = f2.act, -1, 0, _f2i(1.0)
    if f2.drop_id >= 0 and mode == MODE_TRAIN:
        op[O_TBASE], op[O_TCOUNT] = f2.drop_id, _u2i(dropout_threshold(f2.rate))
        op[O_F0] = _f2i(np.float32(1.0) - np.float32(f2.rate))
    op[O_FLAGS], op[O_MODE] = rbw, ncb
    return _fused_program(b, op, 1, 32 * rbw, ncb, mode, n_train, l2c, cin,
                          {'kind': 'mlp2', 'F': F, 'waves': ncb, 'cin': cin, 'act': f1.act, 'act2': f2.act})


RES_NB = (1, 2, 3, 4)    # residual blocks the fused residual-stack kernel is instantiated for
RES_CIN = (88, 96)


def _try_res(b, x_t, y_t, n_train, l2c):
    """Recognise train_88.py's default graph, create_model_complex (Model-88/attention_model.py:97-169)
    and the narrow residual stacks like it: x (88 | 96) -> dense 16 (act, dropout) -> NB x [dense 16
    (act, dropout) -> dense 16 (act, dropout) -> Add(block input) -> act] -> [dense B <= 16 (act,
    dropout)] -> dense 3 (act, dropout); emit a KIND_RES training program for csrc/hpe_res.hip."""
    f = b.fops
    if len(f) < 5 or any(x.kind not in ('dense', 'ew') for x in f):
        return None
    if any(x.kind == 'dense' and (x.transposed or x.w[0] != 'p' or x.act in NEEDS_Z) for x in f):
        return None
    if any(x.bias is not None and x.bias[0] != 'p' for x in f if x.kind == 'dense'):
        return None
    d0 = f[0]
    if d0.kind != 'dense' or d0.ins[0] is not x_t or d0.K not in RES_CIN or d0.N != 16:
        return None
    i, h, nb, post = 1, d0.out, 0, None
    while i + 2 < len(f) and f[i].kind == 'dense' and f[i + 2].kind == 'ew':
        a, c, e = f[i], f[i + 1], f[i + 2]
        if a.ins[0] is not h or a.K != 16 or a.N != 16 or c.kind != 'dense' or c.ins[0] is not a.out:
            return None
        if c.K != 16 or c.N != 16 or len(a.out.consumers) != 1 or len(c.out.consumers) != 1:
            return None
        if e.flags != EW_HAS_B or e.f0 != 1.0 or e.f1 != 1.0 or e.drop_id >= 0 or e.act in NEEDS_Z:
            return None
        if {id(t) for t in e.ins} != {id(h), id(c.out)} or len(e.ins) != 2:
            return None
        if post is not None and e.act != post:
            return None
        post = e.act
        if len(h.consumers) != 2:      # the block's first dense and its Add
            return None
        h, i, nb = e.out, i + 3, nb + 1
    if nb not in RES_NB or len(h.consumers) != 1:
        return None
    rest = f[i:]
    if len(rest) not in (1, 2) or any(x.kind != 'dense' for x in rest):
        return None
    if len(rest) == 2:
        bt, out = rest
        if bt.ins[0] is not h or bt.K != 16 or not 1 <= bt.N <= 16 or out.ins[0] is not bt.out:
            return None
        if len(bt.out.consumers) != 1:
            return None
    else:
        bt, out = None, rest[0]
        if out.ins[0] is not h:
            return None
    if out.out is not y_t or out.N != 3:
        return None

    def ref(r):
        return -1 if r is None else r[1]
    dense = [x for x in f if x.kind == 'dense']
    table = []
    for x in dense:
        ent = [0] * RL_WORDS
        ent[0], ent[1], ent[2] = ref(x.w), ref(x.bias), x.act
        ent[3], ent[4], ent[5] = -1, 0, _f2i(1.0)
        if x.drop_id >= 0:
            ent[3], ent[4] = x.drop_id, _u2i(dropout_threshold(x.rate))
            ent[5] = _f2i(np.float32(1.0) - np.float32(x.rate))
        ent[6], ent[7] = x.K, x.N
        table += ent
    op = [0] * O_WORDS
    op[O_TYPE] = OP_RES
    op[O_K], op[O_N], op[O_AUX3] = d0.K, 16, nb
    op[O_FLAGS] = bt.N if bt is not None else 0
    op[O_MODE] = post
    op[O_AUX0] = H_WORDS + O_WORDS          # the layer table follows the op words
    op[O_AUX1] = len(dense)
    # 512 rows per workgroup: launches of up to 512 rows (every fit batch <= 512) run on ONE
    # workgroup, in the same order as the whole-epoch kernel (bit-identical paths)
    return _fused_program(b, op + table, 3, 512, 8, MODE_TRAIN, n_train, l2c, d0.K,
                          {'kind': 'res', 'blocks': nb, 'bottleneck': bt.N if bt is not None else 0,
                           'layers': len(dense)})


def _fused_program(b, op, kind, T, nw, mode, n_train, l2c, cin, info):
    hdr = [0] * H_WORDS
    hdr[H_MAGIC] = HPE_MAGIC
    hdr[H_NOPS] = 1
    hdr[H_T] = T
    hdr[H_NW] = nw
    hdr[H_CIN], hdr[H_COUT] = cin, 3
    hdr[H_NPARAMS] = n_train + b.const_off
    hdr[H_NPARAMS_TRAIN] = n_train
    hdr[H_MAXACC] = 1
    hdr[H_MAXTHIN] = 1
    hdr[H_SLOTS_OFF] = H_WORDS
    hdr[H_OPS_OFF] = H_WORDS
    hdr[H_MODE] = mode
    hdr[H_SLAB] = -(-(n_train + 4) // 4) * 4
    hdr[H_NPASS] = 1
    hdr[H_GSLOTS] = 0
    hdr[H_KIND] = kind
    words = np.asarray(hdr + op, dtype=np.int64)
    words = ((words + (1 << 31)) % (1 << 32) - (1 << 31)).astype(np.int32)
    prog = Program()
    prog.kind = info['kind']
    prog.words = words
    prog.n_params = n_train + b.const_off
    prog.n_train = n_train
    prog.param_index = {k: b.pidx[k] for k, _ in b.params}
    prog.param_keys = [k for k, _ in b.params]
    prog.consts = np.concatenate(b.consts).astype(np.float32) if b.consts else np.zeros(0, np.float32)
    prog.l2 = np.concatenate(l2c).astype(np.float32) if l2c else np.zeros(0, np.float32)
    prog.mirror = list(b.mirror)
    prog.n_mirror = sum(k * n for _, k, n, _ in b.mirror)
    tpos = np.full(n_train, -1, dtype=np.int32)
    for (o, K, N, mo) in b.mirror:
        if o < n_train:
            idx = np.arange(K * N)
            tpos[o + idx] = mo + (idx % N) * K + idx // N
    prog.tpos = tpos
    prog.T, prog.NW, prog.mode = T, nw, mode
    prog.C_in, prog.C_out = cin, 3
    prog.info = info
    return prog


def _try_chain(b, x_t, y_t, n_train, l2c):
    """Inference chain x -> dense F1 <= 32 -> [dense F2 <= 32] -> dense 3 (e.g. hrchr82r
    96-32-16-3, the selected Model-96 head): KIND_CHAIN program for csrc/hpe_chain.hip."""
    f = b.fops
    if len(f) not in (2, 3) or any(x.kind != 'dense' or x.transposed or x.drop_id >= 0 for x in f):
        return None
    if f[0].ins[0] is not x_t or f[-1].out is not y_t or f[-1].N != 3:
        return None
    for a, c in zip(f, f[1:]):
        if c.ins[0] is not a.out or len(a.out.consumers) != 1:
            return None
    cin = f[0].K
    if cin % 4 or not 80 < cin <= 96 or f[0].N > 32 or (len(f) == 3 and f[1].N > 32):
        return None
    if any(x.act in NEEDS_Z for x in f) or any(x.w[0] != 'p' for x in f):
        return None

    def ref(r):
        if r is None:
            return -1
        return r[1] if r[0] == 'p' else n_train + r[1]
    op = [0] * O_WORDS
    op[O_TYPE] = OP_CHAIN
    op[O_K], op[O_N] = cin, f[0].N
    op[O_W], op[O_BIAS] = ref(f[0].w), ref(f[0].bias)
    op[O_EACT] = f[0].act
    if len(f) == 3:
        op[O_AUX3], op[O_AUX0], op[O_AUX1], op[O_FLAGS] = f[1].N, ref(f[1].w), ref(f[1].bias), f[1].act
    else:
        op[O_AUX3], op[O_AUX0], op[O_AUX1], op[O_FLAGS] = 0, -1, -1, 0
    op[O_AUX2], op[O_TBASE], op[O_MODE], op[O_TCOUNT] = ref(f[-1].w), ref(f[-1].bias), f[-1].act, 3
    op[O_EDROP], op[O_EZ] = -1, -1
    return _fused_program(b, op, 2, 32, 12, MODE_FWD, n_train, l2c, cin,
                          {'kind': 'chain', 'widths': [x.N for x in f]})
