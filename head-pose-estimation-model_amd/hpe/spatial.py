"""Attention heads on H x W > 1 feature maps (SURVEY.md §8 a9 SE block, a10 spatial MHA).

The reference's attention builders (Model-88/attention_model.py:16-72 se_transformer_regr_head,
:74-90 create_modelC) take (batch, H, W, C) maps; the reference trains them on 1x1 maps, where
every op is row-local and the ordinary row program runs them.  On H x W > 1 maps two stages are
not row-local, so the graph is cut there and run as a staged pipeline, every stage on the GPU:

    x --[hpe_se_gate: GAP -> Dense -> Dense -> Multiply, per image]--> xg
      --[row program B: one Dense producing [q/sqrt(d) | k | v]]--> qkv rows
      --[hpe_mha_xg: softmax(q k^T) v per image and head, over the H*W tokens; xg copied
         alongside]--> [xg | o] rows
      --[row program D: attention_output Dense + residual Add + LayerNorm + feed-forward + Add +
         LayerNorm + 1x1-conv regressor, the reference's own layers]--> (yaw, pitch, roll) rows

Programs B and D are ordinary Keras graphs built here from the original layers and weights:
B's kernel is [Wq/sqrt(d) | Wk | Wv]; D reads the [xg | o] row through ONE Dense layer with
kernel [I; Wo] that stands for the residual Add(xg, attention output) (named like the Add; a
graph that reads xg or the attention output elsewhere keeps two Dense layers, [I; 0] and [0; Wo]).  The
Lambda flatten / reshape-back layers are identities on rows.  Forward (predict) only: the
reference trains these heads on 1x1 maps (train_88.py:270-305).
"""
import copy

import numpy as np
import torch

from . import _lib
from .compiler import ACTS, flatten_layers

SPATIAL_OPS = ('GlobalAveragePooling2D', 'MultiHeadAttention')


def is_spatial(model_config):
    layers, _, _ = flatten_layers(model_config)
    return any(l['class_name'] in SPATIAL_OPS for l in layers)


def _ptr(t):
    import ctypes
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream():
    import ctypes
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _layer(cls, name, cfg, ins):
    cfg = dict(cfg, name=name)
    return {'class_name': cls, 'name': name, 'config': cfg,
            'inbound_nodes': [[[i, 0, 0, {}] for i in ins]] if ins else []}


def _input(name, C):
    return _layer('InputLayer', name, {'batch_input_shape': [None, None, None, int(C)],
                                       'dtype': 'float32', 'sparse': False, 'ragged': False}, [])


def _dense(name, units, ins, act='linear'):
    return _layer('Dense', name, {'units': int(units), 'activation': act, 'use_bias': True,
                                  'trainable': True}, ins)


def _model(name, layers, inp, out):
    return {'class_name': 'Functional',
            'config': {'name': name, 'layers': layers, 'input_layers': [[inp, 0, 0]],
                       'output_layers': [[out, 0, 0]]}}


class SpatialPlan:
    """Graph analysis (CPU): the SE parameters, the attention geometry and the two row-local
    sub-graphs (Keras model_config + weights) of a reference attention head."""

    def __init__(self, model_config, weights):
        layers, inp, outs = flatten_layers(model_config)
        if len(outs) != 1:
            raise ValueError('attention heads need a single output')
        by = {l['name']: l for l in layers}
        w = {k: np.asarray(v, dtype=np.float32) for k, v in weights.items()}
        C = int(by[inp]['config']['batch_input_shape'][-1])
        self.C = C
        alias = {}

        def canon(n):
            while n in alias:
                n = alias[n]
            return n
        for l in layers:  # the flatten / reshape-back Lambdas are identities on rows
            if l['class_name'] in ('Lambda', 'Identity'):
                alias[l['name']] = l['ins'][0]
        consumed = {inp}
        # ---- terminal GAP (create_model -> GlobalAveragePooling2D [-> Reshape / Flatten]):
        #      row program on the body, then the per-image mean (hpe_seg_mean) ----
        self.pool = False
        out0 = canon(outs[0])
        tail = by[out0]
        while tail['class_name'] in ('Reshape', 'Flatten') and len(tail['ins']) == 1:
            tail = by[canon(tail['ins'][0])]
        gaps = [l for l in layers if l['class_name'] == 'GlobalAveragePooling2D']
        if tail['class_name'] == 'GlobalAveragePooling2D' and canon(tail['ins'][0]) != inp:
            if len(gaps) != 1 or any(l['class_name'] == 'MultiHeadAttention' for l in layers):
                raise ValueError('terminal GlobalAveragePooling2D with other spatial ops not supported')
            body = []
            for l in layers:
                if l['class_name'] == 'InputLayer':
                    body.append(_input(l['name'], C))
                    continue
                if l['name'] == tail['name']:
                    break
                body.append(_layer(l['class_name'], l['name'], copy.deepcopy(l['config']),
                                   [canon(i) for i in l['ins']]))
            self.pool = True
            self.se = self.mha = None
            self.head_config = _model('spatial_body', body, inp, canon(tail['ins'][0]))
            self.head_weights = dict(w)
            return
        # ---- SE: GAP(x) -> Dense -> Dense -> Reshape -> Multiply(x, .) ----
        self.se = None
        xg = inp
        if gaps:
            if len(gaps) != 1 or canon(gaps[0]['ins'][0]) != inp:
                raise ValueError('SE block: one GlobalAveragePooling2D of the model input expected')
            cons = {}
            for l in layers:
                for i in l['ins']:
                    cons.setdefault(canon(i), []).append(l)
            chain = [gaps[0]]
            for cls in ('Dense', 'Dense', 'Reshape', 'Multiply'):
                nxt = cons.get(chain[-1]['name'], [])
                if len(nxt) != 1 or nxt[0]['class_name'] != cls:
                    raise ValueError('SE block: expected GAP -> Dense -> Dense -> Reshape -> Multiply')
                chain.append(nxt[0])
            d1, d2, mul = chain[1], chain[2], chain[4]
            if sorted(canon(i) for i in mul['ins']) != sorted([inp, chain[3]['name']]):
                raise ValueError('SE block: the gate must multiply the model input')
            U = int(d1['config']['units'])
            if int(d2['config']['units']) != C:
                raise ValueError('SE block: excitation width %d != %d channels' % (d2['config']['units'], C))
            b1 = w.get(d1['name'] + '/bias', np.zeros(U, np.float32))
            b2 = w.get(d2['name'] + '/bias', np.zeros(C, np.float32))
            self.se = dict(U=U, w1=w[d1['name'] + '/kernel'].reshape(C, U), b1=b1,
                           w2=w[d2['name'] + '/kernel'].reshape(U, C), b2=b2,
                           act1=ACTS[d1['config'].get('activation', 'linear')],
                           act2=ACTS[d2['config'].get('activation', 'linear')])
            consumed |= {l['name'] for l in chain}
            xg = mul['name']
        # ---- MHA(flat, flat) ----
        mhas = [l for l in layers if l['class_name'] == 'MultiHeadAttention']
        self.mha = None
        sub_in = 'spatial_in'
        remap = {}
        sub_layers = []
        sub_w = {}
        if mhas:
            if len(mhas) != 1:
                raise ValueError('one MultiHeadAttention layer expected')
            m = mhas[0]
            srcs = [canon(i) for i in m['ins']] + [canon(v) for v in m['kw'].values()]
            if any(s != xg for s in srcs):
                raise ValueError('MultiHeadAttention: self-attention on the (gated) input expected')
            cfg = m['config']
            if cfg.get('attention_axes') not in (None, [1]):
                raise ValueError('MultiHeadAttention: attention over the token axis only')
            H, D = int(cfg['num_heads']), int(cfg['key_dim'])
            if int(cfg.get('value_dim') or D) != D:
                raise ValueError('MultiHeadAttention: value_dim != key_dim not supported')
            HD = H * D
            nm = m['name']

            def mw(part, kind, shape):
                k = '%s/%s/%s' % (nm, part, kind)
                return w[k].reshape(shape) if k in w else np.zeros(shape, np.float32)
            s = np.float32(1.0 / np.sqrt(np.float32(D)))
            wq, wk, wv = (mw(p, 'kernel', (C, HD)) for p in ('query', 'key', 'value'))
            bq, bk, bv = (mw(p, 'bias', (HD,)) for p in ('query', 'key', 'value'))
            wo, bo = mw('attention_output', 'kernel', (HD, C)), mw('attention_output', 'bias', (C,))
            self.mha = dict(H=H, D=D)
            # program B: [q s | k | v] (hpe_mha_xg reads xg from its own rows: no identity block)
            kb = np.concatenate([wq * s, wk, wv], axis=1)
            bb = np.concatenate([bq * s, bk, bv])
            self.qkv_config = _model('spatial_qkv', [_input('qkv_in', C), _dense('qkv', 3 * HD, ['qkv_in'])],
                                     'qkv_in', 'qkv')
            self.qkv_weights = {'qkv/kernel': kb, 'qkv/bias': bb}
            # program D input: [xg | o].  The reference's residual Add(flat, attn) (attention_model.py:
            # 56) reads exactly xg and the attention output, so it folds into ONE Dense with kernel
            # [I; Wo] and bias bo (xg + (o Wo + bo) in one accumulation; no identity GEMM, no Add
            # op); any other reader of xg / the attention output gets [I; 0] / [0; Wo] branches
            res_add = [l for l in layers if l['class_name'] == 'Add' and
                       sorted(canon(i) for i in l['ins']) == sorted([xg, nm])]
            readers = [l for l in layers if l['name'] not in alias and
                       any(canon(i) in (xg, nm) for i in l['ins']) and l['name'] not in
                       {x['name'] for x in res_add} | {nm} | consumed]
            sub_layers.append(_input(sub_in, C + HD))
            if len(res_add) == 1 and not readers:
                fused = res_add[0]['name']
                sub_layers.append(_dense(fused, C, [sub_in]))
                sub_w[fused + '/kernel'] = np.concatenate([np.eye(C, dtype=np.float32), wo])
                sub_w[fused + '/bias'] = bo
                consumed.add(fused)
            else:
                sub_layers += [_dense('spatial_residual', C, [sub_in]), _dense(nm, C, [sub_in])]
                sub_w['spatial_residual/kernel'] = np.concatenate([np.eye(C, dtype=np.float32),
                                                                   np.zeros((HD, C), np.float32)])
                sub_w['spatial_residual/bias'] = np.zeros(C, np.float32)
                sub_w[nm + '/kernel'] = np.concatenate([np.zeros((C, C), np.float32), wo])
                sub_w[nm + '/bias'] = bo
                remap[xg] = 'spatial_residual'
            consumed.add(nm)
            self.d_in = C + HD
        else:
            sub_layers.append(_input(sub_in, C))
            remap[xg] = sub_in
            self.d_in = C
        if xg == inp and self.se is None and self.mha is None:
            raise ValueError('not a spatial attention head')
        # ---- program D: every remaining layer, inputs re-pointed ----
        for l in layers:
            n = l['name']
            if n in consumed or n in alias or l['class_name'] == 'InputLayer' or n == xg:
                continue
            ins = []
            for i in l['ins']:
                ci = canon(i)
                ci = remap.get(ci, ci)
                if ci == inp:
                    raise ValueError('layer %s reads the ungated input: not supported on H x W > 1' % n)
                ins.append(ci)
            if l['kw']:
                raise ValueError('layer %s: keyword inputs not supported' % n)
            cfg = copy.deepcopy(l['config'])
            if l['class_name'] == 'LayerNormalization':
                cfg['axis'] = [3]   # (B, HW, C) axis 2 == channels == NHWC axis 3
            sub_layers.append(_layer(l['class_name'], n, cfg, ins))
            pre = n + '/'
            for k, v in w.items():
                if k.startswith(pre):
                    sub_w[k] = v
        out = canon(outs[0])
        out = remap.get(out, out)
        self.head_config = _model('spatial_head', sub_layers, sub_in, out)
        self.head_weights = sub_w
        self.tail = None
        if self.mha is not None and len(res_add) == 1 and not readers:
            self.tail = _attn_tail(sub_layers, sub_w, C, self.mha['H'] * self.mha['D'], out)


# csrc/hpe_tail.hip descriptor words
(TD_C, TD_HD, TD_FF, TD_HID, TD_ACT_FF, TD_ACT_HID, TD_ACT_OUT, TD_EPS1, TD_EPS2, TD_NW,
 TD_BO, TD_G1, TD_BE1, TD_BF1, TD_BF2, TD_G2, TD_BE2, TD_BC1, TD_BC2) = range(19)
TD_WORDS = 20


def _mfma_order(w, K, N):
    """[K][N] kernel -> the attention-tail kernel's LDS order [K/16][N/16][g][c][s] =
    W[16 bk + 4 g + s][16 bn + c] (zero padded to 16-multiples)."""
    kb, nb = -(-K // 16), -(-N // 16)
    p = np.zeros((kb * 16, nb * 16), np.float32)
    p[:K, :N] = np.asarray(w, np.float32).reshape(K, N)
    return p.reshape(kb, 4, 4, nb, 16).transpose(0, 3, 1, 4, 2).ravel()


def _attn_tail(layers, w, C, HD, out):
    """Recognise program D of se_transformer_regr_head (Model-88/attention_model.py:56-72): the
    [I; Wo] Dense of the residual Add, LayerNorm, Dense(ff) -> Dense(C), Add, LayerNorm, 1x1 conv
    (hidden) -> 1x1 conv (3), and prepare it for csrc/hpe_tail.hip (weights in MFMA order, padded
    vectors, descriptor); None when the graph is anything else."""
    by = {l['name']: l for l in layers}
    ins = {l['name']: [i[0] for i in l['inbound_nodes'][0]] if l['inbound_nodes'] else [] for l in layers}
    cons = {}
    for n, ii in ins.items():
        for i in ii:
            cons.setdefault(i, []).append(n)

    def one(n, cls):
        nx = cons.get(n, [])
        if len(nx) != 1 or by[nx[0]]['class_name'] != cls:
            return None
        return nx[0]
    try:
        seq = [l['name'] for l in layers]
        d0 = seq[1]
        if by[d0]['class_name'] != 'Dense' or by[d0]['config'].get('activation', 'linear') != 'linear':
            return None
        ln1 = one(d0, 'LayerNormalization')
        f1 = [n for n in cons.get(ln1, []) if by[n]['class_name'] == 'Dense']
        add = [n for n in cons.get(ln1, []) if by[n]['class_name'] == 'Add']
        if len(cons.get(ln1, [])) != 2 or len(f1) != 1 or len(add) != 1:
            return None
        f1 = f1[0]
        f2 = one(f1, 'Dense')
        if one(f2, 'Add') != add[0] or sorted(ins[add[0]]) != sorted([ln1, f2]):
            return None
        ln2 = one(add[0], 'LayerNormalization')
        c1 = one(ln2, 'Conv2D')
        c2 = one(c1, 'Conv2D')
        if c2 != out or cons.get(c2):
            return None
    except KeyError:
        return None
    for n in (add[0],):
        if by[n]['config'].get('activation', 'linear') not in (None, 'linear'):
            return None
    for n in (c1, c2):
        cfg = by[n]['config']
        if tuple(cfg.get('kernel_size', (1, 1))) != (1, 1) or tuple(cfg.get('strides', (1, 1))) != (1, 1):
            return None

    def kern(n, K):
        k = np.asarray(w[n + '/kernel'], np.float32)
        return k.reshape(K, -1)

    def vec(n, key, size, fill=0.0):
        k = n + '/' + key
        return np.asarray(w[k], np.float32).ravel() if k in w else np.full(size, fill, np.float32)
    FF = int(by[f1]['config']['units'])
    HID = int(by[c1]['config']['filters'])
    if int(by[f2]['config']['units']) != C or int(by[c2]['config']['filters']) != 3:
        return None
    wo = kern(d0, C + HD)[C:]                    # [I; Wo]: the identity rows are the residual xg
    if not np.array_equal(kern(d0, C + HD)[:C], np.eye(C, dtype=np.float32)):
        return None
    parts = [_mfma_order(wo, HD, C), _mfma_order(kern(f1, C), C, FF), _mfma_order(kern(f2, FF), FF, C),
             _mfma_order(kern(c1, C), C, HID), _mfma_order(kern(c2, HID), HID, 3)]

    def pad(v, n):
        out = np.zeros(-(-n // 16) * 16, np.float32)
        out[:v.size] = v
        return out

    def ln_vec(n, key, fill):
        cfg = by[n]['config']
        on = cfg.get('scale', True) if key == 'gamma' else cfg.get('center', True)
        return vec(n, key, C, fill) if on else np.full(C, fill, np.float32)
    vecs = [('bo', vec(d0, 'bias', C), C), ('g1', ln_vec(ln1, 'gamma', 1.0), C), ('be1', ln_vec(ln1, 'beta', 0.0), C),
            ('bf1', vec(f1, 'bias', FF), FF), ('bf2', vec(f2, 'bias', C), C), ('g2', ln_vec(ln2, 'gamma', 1.0), C),
            ('be2', ln_vec(ln2, 'beta', 0.0), C), ('bc1', vec(c1, 'bias', HID), HID), ('bc2', vec(c2, 'bias', 3), 3)]
    d = np.zeros(TD_WORDS, np.int64)
    off = sum(p.size for p in parts)
    for i, (_, v, n) in enumerate(vecs):
        d[TD_BO + i] = off
        parts.append(pad(v, n))
        off += parts[-1].size
    buf = np.concatenate(parts).astype(np.float32)
    d[TD_C], d[TD_HD], d[TD_FF], d[TD_HID] = C, HD, FF, HID
    d[TD_ACT_FF] = ACTS[by[f1]['config'].get('activation', 'linear')]
    d[TD_ACT_HID] = ACTS[by[c1]['config'].get('activation', 'linear')]
    d[TD_ACT_OUT] = ACTS[by[c2]['config'].get('activation', 'linear')]
    d[TD_EPS1] = np.float32(by[ln1]['config'].get('epsilon', 1e-3)).view(np.int32)
    d[TD_EPS2] = np.float32(by[ln2]['config'].get('epsilon', 1e-3)).view(np.int32)
    d[TD_NW] = buf.size
    return {'desc': d.astype(np.int32), 'w': buf, 'FF': FF, 'HID': HID}


class SpatialHead:
    """Device executor of a SpatialPlan: SE gate kernel, program B, attention kernel, program D."""

    def __init__(self, model_config, weights, device):
        from .engine import Engine
        self.plan = pl = SpatialPlan(model_config, weights)
        self.device = device
        self.C = pl.C
        if pl.pool:
            self.qkv = None
            self.head = Engine(pl.head_config, pl.head_weights, device=device)
            return
        if pl.se is not None:
            self.se = {k: (torch.from_numpy(np.ascontiguousarray(v)).to(device) if isinstance(v, np.ndarray) else v)
                       for k, v in pl.se.items()}
        self.qkv = Engine(pl.qkv_config, pl.qkv_weights, device=device) if pl.mha else None
        self.head = Engine(pl.head_config, pl.head_weights, device=device)
        # the post-attention tail of se_transformer_regr_head in one kernel (csrc/hpe_tail.hip);
        # HPE_ATTN_TAIL=0 keeps the row program D
        self.tail = None
        import os
        if pl.tail is not None and os.environ.get('HPE_ATTN_TAIL', '1') != '0':
            import ctypes
            desc = (ctypes.c_int32 * TD_WORDS)(*[int(v) for v in pl.tail['desc']])
            if _lib.load().hpe_attn_tail_supported(desc) == 1:
                self.tail = {'desc': desc, 'w': torch.from_numpy(pl.tail['w']).to(device)}

    def forward(self, x, P, out=None):
        """x: device fp32 [n_images * P, C] rows -> [n_images * P, C_out]."""
        lib = _lib.load()
        pl = self.plan
        if x.dim() != 2 or x.shape[1] != self.C or x.shape[0] % P:
            raise ValueError('spatial head: expected [n_images*P, %d] rows, got %s' % (self.C, tuple(x.shape)))
        n = x.shape[0] // P
        x = x.contiguous()
        if pl.pool:
            rows = self.head.forward(x, P)
            y = out if out is not None else torch.empty((n, rows.shape[1]), dtype=torch.float32, device=x.device)
            _lib.check(lib.hpe_seg_mean(_ptr(rows), _ptr(y), n, P, rows.shape[1], _stream()), 'hpe_seg_mean')
            return y
        if pl.se is not None:
            xg = torch.empty_like(x)
            s = self.se
            _lib.check(lib.hpe_se_gate(_ptr(x), _ptr(xg), n, P, self.C, _ptr(s['w1']), _ptr(s['b1']), s['U'],
                                       s['act1'], _ptr(s['w2']), _ptr(s['b2']), s['act2'], _stream()),
                       'hpe_se_gate')
        else:
            xg = x
        if pl.mha is None:
            return self.head.forward(xg, P, out=out)
        H, D = pl.mha['H'], pl.mha['D']
        qkv = self.qkv.forward(xg, P)
        if self.tail is not None:
            # attention core writes o alone (no pass-through columns); the tail reads xg and o
            o = torch.empty((x.shape[0], H * D), dtype=torch.float32, device=x.device)
            _lib.check(lib.hpe_mha_xg(_ptr(qkv), qkv.shape[1], _ptr(None), 0, _ptr(o), H * D, n, P, H, D, _stream()),
                       'hpe_mha_xg')
            y = out if out is not None else torch.empty((x.shape[0], 3), dtype=torch.float32, device=x.device)
            _lib.check(lib.hpe_attn_tail(_ptr(xg), self.C, _ptr(o), H * D, x.shape[0], self.tail['desc'],
                                         _ptr(self.tail['w']), _ptr(y), _stream()), 'hpe_attn_tail')
            return y
        xo = torch.empty((x.shape[0], self.C + H * D), dtype=torch.float32, device=x.device)
        _lib.check(lib.hpe_mha_xg(_ptr(qkv), qkv.shape[1], _ptr(xg), self.C, _ptr(xo), xo.shape[1], n, P, H, D,
                                  _stream()), 'hpe_mha_xg')
        return self.head.forward(xo, P, out=out)
