"""BlazeFace + pose-regressor unified graph on the MI355X.

The reference runs the fused detector/regressor Keras graph one frame at a time
(`BlazePoser/blazeFaceDetectorH5.py:272`, graphs built by `JoinModels.py:43-66`); this module reads the
same ``model_config`` (the unified ``.h5`` attr, converted to a fixture), recognises its structure
and lowers it to a plan of fused HIP kernels (``csrc/hpe_blaze.hip``):

    stem     conv 5x5 s2 'same' (3 -> 24) + ReLU
    blocks   DepthwiseConv2D 3x3 (s1|s2) -> 1x1 conv -> + residual (x, or MaxPool 2x2 then zero
             channel Pad) -> ReLU, one kernel per block
    heads    the 1x1 detector convs on each tap, paired into one GEMM with a split epilogue
    pose     the two embedded regressors (``model`` on re_lu_10, ``model_10`` on re_lu_15) through
             the row-program engine (hpe_forward) at P = 16*16 and 8*8

Outputs are returned in the unified model's ``output_layers`` order, as Keras' ``predict`` does.
"""
import ctypes

import numpy as np
import torch

from . import _lib

BF_MAGIC = 0x46425048
BFH_WORDS = 8
(BFH_MAGIC, BFH_NOPS, BFH_ACT_FLOATS, BFH_OPS_OFF) = range(4)
BF_STEM, BF_BLOCK, BF_ROWS, BF_DIRECT, BF_STAGE, BF_FRONT = 1, 2, 3, 4, 5, 6
# 8x8 maps and the detector heads: persistent direct-tap kernel (HPE_BF_DIRECT=0 -> tiles); the
# 16x16 maps measured equal either way and keep the tile kernel
import os as _os
USE_DIRECT = _os.environ.get('HPE_BF_DIRECT', '1') != '0'
DIRECT_MAX_WO = int(_os.environ.get('HPE_BF_DIRECT_MAX_WO', '8'))
ROWS_MIN_WO = int(_os.environ.get('HPE_BF_ROWS_MIN_WO', '32'))   # row-streaming kernel from this width


def _direct(f, dw, cinp, nct, ks):
    """Words of the persistent direct-tap kernel (csrc/hpe_blaze.hip bf_direct_kernel)."""
    f[BFO_KIND] = BF_DIRECT
    f[BFO_TH], f[BFO_NI], f[BFO_ROWS], f[BFO_COLS] = f[BFO_HO], 1, 0, 0
    f[BFO_CS], f[BFO_KS], f[BFO_NC], f[BFO_NCT], f[BFO_WAVES] = ks, ks, nct, nct, 4
    f[BFO_LDS] = 4 * (nct * 32 * ks + (10 * cinp if dw else 0))
ROWS_PF = 4                 # float4 per thread the rows kernel prefetches per step (csrc RPF)
# stage (csrc bf_stage_kernel): the blocks on maps of <= STAGE_MAX_HW positions and the detector
# heads as one launch, one 8-wave workgroup per image, the map resident in LDS
STAGE_MAX_HW, STAGE_NW, STAGE_PF, STAGE_MAXNC = 256, 8, 6, 3
RES_NONE, RES_ID, RES_MAXPOOL = 0, 1, 2
BUF_IMG, BUF_A, BUF_B, BUF_OUT0 = 0, 1, 2, 3
(BFO_KIND, BFO_H, BFO_W, BFO_HO, BFO_WO, BFO_CIN, BFO_COUT, BFO_CINP, BFO_COUTP,
 BFO_STRIDE, BFO_PADT, BFO_PADL, BFO_DW, BFO_RES, BFO_RELU, BFO_SRC, BFO_DST, BFO_DST2,
 BFO_SPLIT, BFO_TH, BFO_NI, BFO_DWW, BFO_PWW, BFO_PWB, BFO_CS, BFO_KS, BFO_ROWS, BFO_COLS,
 BFO_NC, BFO_LDS, BFO_OSTRIDE, BFO_NCT, BFO_WAVES) = range(33)
BFO_WORDS = 40
STEM_TH = 4


def _r8(c):
    return (c + 7) // 8 * 8


def _same_pad(n, k, s):
    """TF 'same' padding (before, after) of one spatial dim."""
    out = -(-n // s)
    total = max((out - 1) * s + k - n, 0)
    return total // 2, total - total // 2


# ------------------------------------------------------------------------------------------------
# structure recognition
# ------------------------------------------------------------------------------------------------
def _graph(mc):
    cfg = mc.get('config', mc)
    layers = {l['name']: l for l in cfg['layers']}
    ins = {n: [t[0] for node in l.get('inbound_nodes') or [] for t in node] for n, l in layers.items()}
    cons = {n: [] for n in layers}
    for n, src in ins.items():
        for s in src:
            cons[s].append(n)
    return cfg, layers, ins, cons


def is_blazeface(model_config):
    cfg = model_config.get('config', model_config)
    return any(l['class_name'] == 'DepthwiseConv2D' for l in cfg['layers'])


def parse(model_config):
    """Unified BlazeFace graph -> dict(stem, blocks, heads, regressors, outputs, input_hw).
    Raises ValueError on any deviation from the structure the kernels implement."""
    cfg, layers, ins, cons = _graph(model_config)
    inp = cfg['input_layers'][0][0]
    shp = layers[inp]['config']['batch_input_shape']
    H, W, C = shp[1], shp[2], shp[3]
    if C != 3 or H is None or W is None:
        raise ValueError('BlazeFace input must be (H, W, 3) with static H, W; got %s' % (shp,))

    def only(lst, what):
        if len(lst) != 1:
            raise ValueError('BlazeFace graph: expected one %s, found %s' % (what, lst))
        return lst[0]

    def cls(n):
        return layers[n]['class_name']

    def conf(n):
        return layers[n]['config']

    stem = only([n for n in cons[inp] if cls(n) == 'Conv2D'], 'stem conv')
    sc = conf(stem)
    if (tuple(sc['kernel_size']) != (5, 5) or tuple(sc['strides']) != (2, 2) or sc['padding'] != 'same'
            or sc['activation'] != 'relu' or not sc.get('use_bias', True)):
        raise ValueError('BlazeFace stem must be conv 5x5 s2 same relu: %s' % sc)
    blocks = []
    cur, h, w, c = stem, -(-H // 2), -(-W // 2), sc['filters']
    shapes = {stem: (h, w, c)}
    while True:
        dws = [n for n in cons[cur] if cls(n) == 'DepthwiseConv2D']
        if not dws:
            break
        dw = only(dws, 'depthwise conv')
        dc = conf(dw)
        s = dc['strides'][0]
        if (tuple(dc['kernel_size']) != (3, 3) or dc['strides'][0] != dc['strides'][1] or s not in (1, 2)
                or dc['padding'] != 'same' or dc['activation'] != 'linear' or dc.get('depth_multiplier', 1) != 1
                or not dc.get('use_bias', True)):
            raise ValueError('depthwise %s: only 3x3 s1/s2 same linear (+bias) supported' % dw)
        pw = only(cons[dw], 'pointwise after %s' % dw)
        pc = conf(pw)
        if cls(pw) != 'Conv2D' or tuple(pc['kernel_size']) != (1, 1) or pc['activation'] != 'linear' \
                or tuple(pc['strides']) != (1, 1) or not pc.get('use_bias', True):
            raise ValueError('block after %s: expected a linear 1x1 conv, got %s' % (dw, pw))
        add = only(cons[pw], 'Add after %s' % pw)
        if cls(add) != 'Add' or len(ins[add]) != 2:
            raise ValueError('block %s: expected Add' % pw)
        other = [x for x in ins[add] if x != pw]
        other = other[0]
        res, pad = None, 0
        if other == cur:
            res = RES_ID
        elif cls(other) == 'TensorFlowOpLayer' and conf(other)['node_def']['op'] == 'Pad':
            pads = conf(other)['constants']['1']
            if any(p != [0, 0] for p in pads[:3]) or pads[3][0] != 0:
                raise ValueError('residual Pad %s: only trailing channel padding supported' % other)
            pad = pads[3][1]
            src = only(ins[other], 'Pad input')
            if src == cur:
                res = RES_ID
            elif cls(src) == 'MaxPooling2D' and ins[src] == [cur]:
                mp = conf(src)
                if tuple(mp['pool_size']) != (2, 2) or tuple(mp['strides']) != (2, 2):
                    raise ValueError('maxpool %s: only 2x2 s2' % src)
                res = RES_MAXPOOL
            else:
                raise ValueError('residual %s: unsupported source %s' % (other, src))
        elif cls(other) == 'MaxPooling2D' and ins[other] == [cur]:
            res = RES_MAXPOOL
        else:
            raise ValueError('block %s: unsupported residual %s' % (add, other))
        if (res == RES_MAXPOOL) != (s == 2):
            raise ValueError('block %s: stride-2 blocks need the MaxPool residual and vice versa' % dw)
        if s == 2 and (h % 2 or w % 2):
            raise ValueError('block %s: stride 2 on an odd map' % dw)
        relu = only(cons[add], 'ReLU after %s' % add)
        rc = conf(relu)
        if cls(relu) != 'ReLU' or rc.get('max_value') is not None or float(rc.get('negative_slope', 0)) != 0 \
                or float(rc.get('threshold', 0)) != 0:
            raise ValueError('block %s: expected plain ReLU' % add)
        cout = pc['filters']
        if cout != c + pad:
            raise ValueError('block %s: residual channels %d + pad %d != %d' % (add, c, pad, cout))
        ho, wo = (h, w) if s == 1 else (h // 2, w // 2)
        blocks.append(dict(dw=dw, pw=pw, out=relu, src=cur, stride=s, res=res, H=h, W=w, Ho=ho, Wo=wo,
                           cin=c, cout=cout))
        cur, h, w, c = relu, ho, wo, cout
        shapes[relu] = (h, w, c)
    outs = [t[0] for t in cfg['output_layers']]
    heads, regs = [], []
    for o in outs:
        oc = cls(o)
        if oc == 'TensorFlowOpLayer' and conf(o)['node_def']['op'] == 'Reshape':
            conv = only(ins[o], 'head conv')
            cc = conf(conv)
            tap = only(ins[conv], 'head input')
            if cls(conv) != 'Conv2D' or tuple(cc['kernel_size']) != (1, 1) or cc['activation'] != 'linear' \
                    or tap not in shapes or tap == stem:
                raise ValueError('output %s: expected Reshape(linear 1x1 conv(block output))' % o)
            tshape = [int(v) for v in conf(o)['constants']['1']][1:]
            th_, tw_, _ = shapes[tap]
            if int(np.prod(tshape)) != th_ * tw_ * cc['filters']:
                raise ValueError('output %s: Reshape %s does not match %s' % (o, tshape, (th_, tw_, cc['filters'])))
            heads.append(dict(out=o, conv=conv, tap=tap, n=cc['filters'], shape=tuple(tshape)))
        elif oc == 'Functional':
            rs = only(ins[o], 'regressor input')
            tap = rs
            if cls(rs) == 'Reshape':
                tap = only(ins[rs], 'reshape input')
                if tuple(conf(rs)['target_shape']) != tuple(shapes.get(tap, ())):
                    raise ValueError('regressor %s: Reshape changes the tap shape' % o)
            if tap not in shapes or tap == stem:
                raise ValueError('regressor %s: input is not a block output' % o)
            regs.append(dict(out=o, tap=tap, config=layers[o]['config']))
        else:
            raise ValueError('unsupported unified-model output %s (%s)' % (o, oc))
    taps = []
    for t in [x['tap'] for x in heads] + [x['tap'] for x in regs]:
        if t not in taps:
            taps.append(t)
    return dict(input_hw=(H, W), stem=stem, stem_cout=sc['filters'], blocks=blocks, heads=heads,
                regressors=regs, outputs=outs, taps=taps, shapes=shapes)


# ------------------------------------------------------------------------------------------------
# plan (op words + flat padded parameters)
# ------------------------------------------------------------------------------------------------
class _Params:
    def __init__(self):
        self.chunks, self.n = [], 0

    def add(self, a):
        a = np.ascontiguousarray(a, dtype=np.float32).ravel()
        off = self.n
        pad = (-a.size) % 4                     # keep every table 16-B aligned
        self.chunks.append(np.concatenate([a, np.zeros(pad, np.float32)]))
        self.n += a.size + pad
        return off

    def flat(self):
        return np.concatenate(self.chunks) if self.chunks else np.zeros(0, np.float32)


def _block_tile(ho, wo, s, dw, cinp, nct, ks, cs):
    """Pick the tile (TH rows of one image, or NI whole images), the output-channel chunks per wave
    task (NC) and the waves per workgroup: maximise resident waves per CU (LDS-limited, capped at
    16), then minimise the halo re-read factor, then prefer more channel chunks per task (no
    depthwise recompute).  Wo and TH*Wo must be powers of two (kernel uses shifts)."""
    best = None
    cands = [(th, 1) for th in range(1, ho + 1) if ho % th == 0] + [(ho, ni) for ni in (2, 4, 8)]
    for th, ni in cands:
        npos = ni * th * wo
        ppi = th * wo
        if npos % 32 or npos > 512 or (ppi & (ppi - 1)) or (wo & (wo - 1)):
            continue
        rows = (th - 1) * s + 3 if dw else th
        cols = (wo - 1) * s + 3 if dw else wo
        lds = 4 * (nct * 32 * ks + (10 * cinp if dw else 0) + ni * rows * cols * cs)
        if lds > 160 * 1024:
            continue
        for nc in [d for d in (1, 2, 3, 4) if nct % d == 0]:
            tasks = (npos // 32) * (nct // nc)
            waves = min(tasks, 8)
            if cinp // 4 > 64 * waves:
                continue
            vg_waves = 8 if nc <= 2 else 5            # waves/SIMD the VGPR budget allows
            per_cu = min((160 * 1024) // lds * waves, 4 * vg_waves, 16)
            halo = rows * cols / float(th * wo * s * s)
            key = (per_cu, -round(halo, 3), nc)
            if best is None or key > best[0]:
                best = (key, th, ni, rows, cols, lds, nc, waves)
    if best is None:
        raise ValueError('no BlazeFace tile fits LDS for %dx%d Cin %d' % (ho, wo, cinp))
    return best[1:]


def _rows_plan(bl, cinp, nct, ks, cs):
    """Row-streaming variant for the large maps: steps of R output rows (R*Wo = 128 positions
    when the per-thread prefetch share allows), 4 waves, NSEG segments per image."""
    s, wo, w, ho = bl['stride'], bl['Wo'], bl['W'], bl['Ho']
    kq = cinp // 4
    for r in (128 // wo, 64 // wo, 32 // wo):
        if r < 1 or ho % r or (r * wo) % 32:
            continue
        if r * s * w * kq > ROWS_PF * 256:
            continue
        ring, cols = (r - 1) * s + 3, (wo - 1) * s + 3
        nc = nct if nct <= 2 else 1
        lds = 4 * (nct * 32 * ks + 10 * cinp + ring * cols * cs)
        if lds > 160 * 1024:
            continue
        steps = ho // r
        nseg = 2 if steps % 2 == 0 and steps >= 8 else 1
        return r, nseg, ring, cols, lds, nc, 4
    return None


def _stage_nc(nchunk, nct):
    """csrc bfs_nc: fewest output-channel chunks per wave task with every task on its own wave."""
    for nc in range(1, min(nct, STAGE_MAXNC) + 1):
        if nct % nc == 0 and nchunk * (nct // nc) <= STAGE_NW:
            return nc
    return 0


def _stage_record(recs):
    """BF_STAGE record for the op records `recs` (blocks, each tap's heads right after it), or None
    when they do not fit the stage kernel (map / channel geometry, LDS)."""
    for k, f in enumerate(recs):
        hw, wo, dw = f[BFO_HO] * f[BFO_WO], f[BFO_WO], f[BFO_DW]
        if hw > STAGE_MAX_HW or hw % 32 or wo & (wo - 1) or f[BFO_NCT] > 4 or not _stage_nc(hw // 32, f[BFO_NCT]):
            return None
        if (f[BFO_COUTP] + (10 if dw else 0)) * (f[BFO_CINP] // 4) > STAGE_PF * STAGE_NW * 64:
            return None
        if k == 0 and not dw:
            return None
    blocks = [f for f in recs if f[BFO_DW]]
    cs = max(f[BFO_COUTP] for f in blocks) + 4           # (cs / 4) odd: conflict-free b128 rows
    # each resident map: a zero row above and below, channel stride coutp + 4 of its writer
    mapf = max((f[BFO_HO] + 2) * f[BFO_WO] * (f[BFO_COUTP] + 4) for f in blocks)
    wtf = max(f[BFO_COUTP] * f[BFO_KS] for f in recs)
    dwf = max(10 * f[BFO_CINP] for f in blocks)
    lds = 4 * (mapf + wtf + dwf)
    if lds > 160 * 1024:
        return None
    f = [0] * BFO_WORDS
    f[BFO_KIND], f[BFO_NI], f[BFO_CS], f[BFO_ROWS], f[BFO_COLS] = BF_STAGE, len(recs), cs, mapf, wtf
    f[BFO_LDS], f[BFO_WAVES] = lds, STAGE_NW
    return f


def _with_stage(stem_op, block_ops, head_ops):
    """Op list with the longest stage-able suffix of the blocks (and every detector head, placed
    right after the block that produces its tap) behind one BF_STAGE record; the per-op list when
    no suffix qualifies."""
    heads_of = {}
    for f in head_ops:
        heads_of.setdefault(f[BFO_SRC], []).append(f)
    for b0 in range(len(block_ops)):
        suffix = block_ops[b0:]
        if any(f[BFO_HO] * f[BFO_WO] > STAGE_MAX_HW for f in suffix):
            continue
        recs, placed = [], 0
        for f in suffix:
            recs.append(f)
            for h in heads_of.get(f[BFO_DST], []) if f[BFO_DST] >= BUF_OUT0 else []:
                recs.append(h)
                placed += 1
        if placed != len(head_ops) or len(recs) > 16:
            continue
        rec = _stage_record(recs)
        if rec is not None:
            return [stem_op] + block_ops[:b0] + [rec] + recs
    return [stem_op] + block_ops + head_ops


# front (csrc bf_front_kernel): the stem and the first five blocks of the BlazeFace backbone as ONE
# launch, the maps streamed through LDS rings; its geometry is fixed in the kernel (BffL)
FRONT_LDS = 4 * 40504
_FRONT_BLOCKS = [(1, 24, 24, 64, 64, 1, RES_ID), (1, 24, 32, 64, 64, 1, RES_ID), (2, 32, 32, 64, 32, 0, RES_MAXPOOL),
                 (1, 32, 40, 32, 32, 1, RES_ID), (1, 40, 48, 32, 32, 1, RES_ID)]


def _with_front(ops):
    """A BF_FRONT record ahead of the stem and the first five blocks when they are the backbone
    bf_front_kernel implements (csrc check_front); the op list unchanged otherwise."""
    if len(ops) < 6:
        return ops
    g = ops[0]
    if (g[BFO_KIND] != BF_STEM or (g[BFO_H], g[BFO_W], g[BFO_HO], g[BFO_WO], g[BFO_COUT], g[BFO_STRIDE],
                                   g[BFO_PADT], g[BFO_PADL], g[BFO_SRC]) != (128, 128, 64, 64, 24, 2, 1, 1, BUF_IMG)):
        return ops
    last = g[BFO_DST]
    if last not in (BUF_A, BUF_B):       # the front keeps the stem's map in LDS only
        return ops
    for b, (s, cinp, coutp, h, ho, pad, res) in zip(ops[1:6], _FRONT_BLOCKS):
        if (b[BFO_KIND] not in (BF_ROWS, BF_BLOCK) or not b[BFO_DW] or not b[BFO_RELU] or b[BFO_SPLIT] or
                (b[BFO_STRIDE], b[BFO_CINP], b[BFO_COUTP], b[BFO_H], b[BFO_W], b[BFO_HO], b[BFO_WO], b[BFO_PADT],
                 b[BFO_PADL], b[BFO_RES], b[BFO_OSTRIDE]) != (s, cinp, coutp, h, h, ho, ho, pad, pad, res, coutp)
                or b[BFO_SRC] != last):
            return ops
        last = b[BFO_DST]
        if last not in (BUF_A, BUF_B):   # blocks 1-4: LDS only; block 5: the workspace map it writes
            return ops
    # the record after the front must read block 5's map (the others never reach HBM)
    nxt = ops[6] if len(ops) > 6 else None
    if nxt is not None:
        rec = ops[7] if nxt[BFO_KIND] == BF_STAGE and len(ops) > 7 else nxt
        if rec[BFO_SRC] != last:
            return ops
    f = [0] * BFO_WORDS
    f[BFO_KIND], f[BFO_NI], f[BFO_LDS] = BF_FRONT, 6, FRONT_LDS
    return [f] + ops


def build_plan(model_config, weights, stage=None, front=None):
    """Plan words + packed parameters.  stage: run the small-map blocks and the heads as one
    bf_stage_kernel launch (default: env HPE_BF_STAGE, on); front: the stem and the 64x64 / 32x32
    blocks as one bf_front_kernel launch (default: env HPE_BF_FRONT, on)."""
    if stage is None:
        stage = _os.environ.get('HPE_BF_STAGE', '1') != '0'
    if front is None:
        front = _os.environ.get('HPE_BF_FRONT', '1') != '0'
    st = parse(model_config)
    P = _Params()
    ops = []
    H, W = st['input_hw']
    wk = lambda layer, var: np.asarray(weights['%s/%s' % (layer, var)], np.float32)

    # stem: W^T [32][90], k = (ky*5 + kx)*3 + c over a 6-row window (row 5 zero)
    k = wk(st['stem'], 'kernel')                    # (5,5,3,24) HWIO
    cout = k.shape[3]
    if cout > 32:
        raise ValueError('stem with %d filters > 32' % cout)
    wt = np.zeros((32, 6, 5, 3), np.float32)
    wt[:cout, :5] = np.transpose(k, (3, 0, 1, 2))
    b = np.zeros(32, np.float32)
    b[:cout] = wk(st['stem'], 'bias')
    pwb = P.add(b)
    pww = P.add(wt.reshape(32, 90))
    ho, wo = -(-H // 2), -(-W // 2)
    pt, _ = _same_pad(H, 5, 2)
    pl, _ = _same_pad(W, 5, 2)
    if ho % STEM_TH or (STEM_TH * wo) % 32:
        raise ValueError('stem output %dx%d does not tile by %d rows' % (ho, wo, STEM_TH))
    f = [0] * BFO_WORDS
    rows, cols = 2 * (STEM_TH - 1) + 6, 2 * (wo - 1) + 5
    f[BFO_KIND], f[BFO_H], f[BFO_W], f[BFO_HO], f[BFO_WO] = BF_STEM, H, W, ho, wo
    f[BFO_CIN], f[BFO_COUT], f[BFO_CINP], f[BFO_COUTP] = 3, cout, 3, _r8(cout)
    f[BFO_STRIDE], f[BFO_PADT], f[BFO_PADL] = 2, pt, pl
    f[BFO_SRC], f[BFO_DST] = BUF_IMG, BUF_A
    f[BFO_TH], f[BFO_NI], f[BFO_PWW], f[BFO_PWB] = STEM_TH, 1, pww, pwb
    f[BFO_ROWS], f[BFO_COLS], f[BFO_NC], f[BFO_LDS] = rows, cols, 1, rows * cols * 12
    f[BFO_NCT], f[BFO_WAVES] = 1, min(4, STEM_TH * wo // 32)
    if _r8(cout) != cout:
        raise ValueError('stem filters %d: multiple of 8 required' % cout)
    ops.append(f)
    act_floats = ho * wo * _r8(cout)

    # blocks; taps go to the caller's output buffers 4 (first tap) and 5 (second)
    tap_buf = {t: BUF_OUT0 + 4 + i for i, t in enumerate(st['taps'])}
    if len(st['taps']) > 2:
        raise ValueError('more than two taps')
    cur_buf = BUF_A
    for bi, bl in enumerate(st['blocks']):
        cin, cout = bl['cin'], bl['cout']
        cinp, coutp = _r8(cin), _r8(cout)
        dk = wk(bl['dw'], 'depthwise_kernel')[:, :, :, 0]      # (3,3,Cin)
        tab = np.zeros((10, cinp), np.float32)
        tab[:9, :cin] = dk.reshape(9, cin)
        tab[9, :cin] = wk(bl['dw'], 'bias')
        dww = P.add(tab)
        pk = wk(bl['pw'], 'kernel')[0, 0]                     # (Cin, Cout)
        wt = np.zeros((coutp, cinp), np.float32)
        wt[:cout, :cin] = pk.T
        pww = P.add(wt)
        bb = np.zeros(coutp, np.float32)
        bb[:cout] = wk(bl['pw'], 'bias')
        pwb = P.add(bb)
        nct = -(-coutp // 32)
        s = bl['stride']
        cs = ks = cinp + 4                                    # (cs/4) odd: conflict-free b128 rows
        rows_plan = _rows_plan(bl, cinp, nct, ks, cs) if bl['Wo'] >= ROWS_MIN_WO else None
        if rows_plan:
            th, ni, rows, cols, lds, nc, waves = rows_plan
        else:
            th, ni, rows, cols, lds, nc, waves = _block_tile(bl['Ho'], bl['Wo'], s, True, cinp, nct, ks, cs)
        if bl['out'] in tap_buf:
            dst = tap_buf[bl['out']]
            if coutp != cout:
                raise ValueError('tap %s has %d channels (multiple of 8 required)' % (bl['out'], cout))
        else:
            dst = BUF_B if cur_buf == BUF_A else BUF_A
        f = [0] * BFO_WORDS
        f[BFO_KIND] = BF_ROWS if rows_plan else BF_BLOCK
        f[BFO_H], f[BFO_W], f[BFO_HO], f[BFO_WO] = bl['H'], bl['W'], bl['Ho'], bl['Wo']
        f[BFO_CIN], f[BFO_COUT], f[BFO_CINP], f[BFO_COUTP] = cin, cout, cinp, coutp
        f[BFO_STRIDE] = s
        f[BFO_PADT], f[BFO_PADL] = (1, 1) if s == 1 else (0, 0)
        f[BFO_DW], f[BFO_RES], f[BFO_RELU] = 1, bl['res'], 1
        f[BFO_SRC], f[BFO_DST] = cur_buf, dst
        f[BFO_TH], f[BFO_NI], f[BFO_DWW], f[BFO_PWW], f[BFO_PWB] = th, ni, dww, pww, pwb
        f[BFO_CS], f[BFO_KS], f[BFO_ROWS], f[BFO_COLS], f[BFO_NC], f[BFO_LDS] = cs, ks, rows, cols, nc, lds
        f[BFO_OSTRIDE], f[BFO_NCT], f[BFO_WAVES] = coutp, nct, waves
        if not rows_plan and USE_DIRECT and nct <= 4 and bl["Wo"] <= DIRECT_MAX_WO:
            _direct(f, True, cinp, nct, ks)
        ops.append(f)
        if dst in (BUF_A, BUF_B):
            act_floats = max(act_floats, bl['Ho'] * bl['Wo'] * coutp)
        cur_buf = dst

    # heads: per tap, up to two 1x1 convs fused into one GEMM with a split epilogue
    out_index = {o: i for i, o in enumerate(st['outputs'])}
    det_outs = [h['out'] for h in st['heads']]
    det_slot = {o: BUF_OUT0 + i for i, o in enumerate(det_outs)}
    for tap in st['taps']:
        hs = [h for h in st['heads'] if h['tap'] == tap]
        if not hs:
            continue
        if len(hs) > 2:
            raise ValueError('more than two detector heads on %s' % tap)
        th_, tw_, cin = st['shapes'][tap]
        cinp = _r8(cin)
        ns = [h['n'] for h in hs]
        cout = sum(ns)
        coutp = _r8(cout)
        wt = np.zeros((coutp, cinp), np.float32)
        bb = np.zeros(coutp, np.float32)
        o = 0
        for h in hs:
            wt[o:o + h['n'], :cin] = wk(h['conv'], 'kernel')[0, 0].T
            bb[o:o + h['n']] = wk(h['conv'], 'bias')
            o += h['n']
        pww, pwb = P.add(wt), P.add(bb)
        nct = -(-coutp // 32)
        if nct > 4:
            raise ValueError('detector heads on %s: %d channels > 128' % (tap, cout))
        cs = ks = cinp + 4
        th, ni, rows, cols, lds, nc, waves = _block_tile(th_, tw_, 1, False, cinp, nct, ks, cs)
        f = [0] * BFO_WORDS
        f[BFO_KIND], f[BFO_H], f[BFO_W], f[BFO_HO], f[BFO_WO] = BF_BLOCK, th_, tw_, th_, tw_
        f[BFO_CIN], f[BFO_COUT], f[BFO_CINP], f[BFO_COUTP] = cin, cout, cinp, coutp
        f[BFO_STRIDE], f[BFO_DW], f[BFO_RES], f[BFO_RELU] = 1, 0, RES_NONE, 0
        f[BFO_SRC], f[BFO_DST] = tap_buf[tap], det_slot[hs[0]['out']]
        if len(hs) == 2:
            f[BFO_SPLIT], f[BFO_DST2] = ns[0], det_slot[hs[1]['out']]
        else:
            f[BFO_SPLIT], f[BFO_DST2], f[BFO_OSTRIDE] = 0, -1, cout
        f[BFO_TH], f[BFO_NI], f[BFO_PWW], f[BFO_PWB] = th, ni, pww, pwb
        f[BFO_CS], f[BFO_KS], f[BFO_ROWS], f[BFO_COLS], f[BFO_NC], f[BFO_LDS] = cs, ks, rows, cols, nc, lds
        f[BFO_NCT], f[BFO_WAVES] = nct, waves
        if USE_DIRECT:
            _direct(f, False, cinp, nct, ks)
        ops.append(f)
    if stage:
        ops = _with_stage(ops[0], ops[1:1 + len(st['blocks'])], ops[1 + len(st['blocks']):])
    if front:
        ops = _with_front(ops)
    hdr = [0] * BFH_WORDS
    hdr[BFH_MAGIC], hdr[BFH_NOPS], hdr[BFH_ACT_FLOATS], hdr[BFH_OPS_OFF] = BF_MAGIC, len(ops), act_floats, BFH_WORDS
    words = np.asarray(hdr + [x for f in ops for x in f], dtype=np.int64)
    if words.max() >= 2 ** 31:
        raise ValueError('plan word overflow')
    return dict(words=words.astype(np.int32), params=P.flat(), structure=st, det_outs=det_outs,
                out_index=out_index)


# ------------------------------------------------------------------------------------------------
# device runner
# ------------------------------------------------------------------------------------------------
def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


class BlazeFace:
    """Batched forward of the unified BlazeFace + regressor graph.  ``predict(images)`` returns
    the unified model's outputs (Keras order) as numpy arrays; ``forward`` keeps them on device."""

    def __init__(self, model_config, weights, device=None, stage=None, front=None):
        if not torch.cuda.is_available():
            raise _lib.HPEError('hpe needs a ROCm GPU (MI355X / gfx950); torch.cuda is unavailable')
        from .engine import Engine
        self.device = torch.device(device or 'cuda')
        self.plan = build_plan(model_config, weights, stage=stage, front=front)
        st = self.plan['structure']
        lib = _lib.load()
        h = ctypes.c_void_p()
        w = np.ascontiguousarray(self.plan['words'], np.int32)
        _lib.check(lib.hpe_blazeface_create(w.ctypes.data_as(ctypes.c_void_p), w.size, ctypes.byref(h)),
                   'hpe_blazeface_create')
        self.h = h
        self.params = torch.from_numpy(self.plan['params']).to(self.device)
        self.ws = None
        self.regs = []
        for r in st['regressors']:
            prefix = r['out'] + '/'
            sub = {k[len(prefix):]: v for k, v in weights.items() if k.startswith(prefix)}
            eng = Engine({'class_name': 'Functional', 'config': r['config']}, sub, device=self.device)
            self.regs.append((r, eng))
        self.structure = st

    def __del__(self):
        try:
            if getattr(self, 'h', None):
                _lib.load().hpe_blazeface_destroy(self.h)
        except Exception:
            pass

    def output_shapes(self, n):
        st = self.structure
        shp = {}
        for hd in st['heads']:
            shp[hd['out']] = (n,) + hd['shape']
        for r, _ in self.regs:
            th, tw, _ = st['shapes'][r['tap']]
            shp[r['out']] = (n, th, tw, 3)
        return shp

    def forward(self, images):
        """images: device fp32 (n, H, W, 3).  Returns the list of device outputs (Keras order)."""
        st = self.structure
        x = images.contiguous()
        H, W = st['input_hw']
        if x.dim() != 4 or tuple(x.shape[1:]) != (H, W, 3):
            raise ValueError('BlazeFace input must be (n, %d, %d, 3), got %s' % (H, W, tuple(x.shape)))
        if x.dtype != torch.float32:
            raise ValueError('BlazeFace input must be float32')
        n = x.shape[0]
        lib = _lib.load()
        need = lib.hpe_blazeface_workspace_size(self.h, n)
        if self.ws is None or self.ws.numel() * 4 < need:
            self.ws = torch.empty(max(need // 4, 4), dtype=torch.float32, device=self.device)
        shapes = self.output_shapes(n)
        det = [torch.empty(shapes[o], dtype=torch.float32, device=self.device) for o in self.plan['det_outs']]
        while len(det) < 4:
            det.append(torch.empty(4, dtype=torch.float32, device=self.device))
        taps = []
        for t in st['taps']:
            th, tw, c = st['shapes'][t]
            taps.append(torch.empty((n, th, tw, c), dtype=torch.float32, device=self.device))
        while len(taps) < 2:
            taps.append(torch.empty(4, dtype=torch.float32, device=self.device))
        bufs = det + taps
        arr = (ctypes.c_void_p * 6)(*[b.data_ptr() for b in bufs])
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        _lib.check(lib.hpe_blazeface_forward(self.h, _ptr(self.params), _ptr(x), n, arr, _ptr(self.ws),
                                             stream), 'hpe_blazeface_forward')
        res = {o: det[i] for i, o in enumerate(self.plan['det_outs'])}
        for r, eng in self.regs:
            tap = taps[st['taps'].index(r['tap'])]
            th, tw, c = st['shapes'][r['tap']]
            y = eng.forward(tap.view(n * th * tw, c), th * tw)
            res[r['out']] = y.view(n, th, tw, 3)
        self.taps = {t: taps[i] for i, t in enumerate(st['taps'])}
        return [res[o] for o in st['outputs']]

    def predict(self, images, batch_size=None):
        x = torch.as_tensor(np.ascontiguousarray(images, np.float32)).to(self.device)
        outs = self.forward(x)
        return [o.cpu().numpy() for o in outs]


def work_per_image(plan):
    """Algorithmic work of one 128x128 frame through the plan: FLOP = 2*MAC of the
    convs (depthwise, pointwise, stem, heads) and the regressors; bytes = the PLAN's traffic (each
    launch's input and output maps, not the frame's compulsory bytes: compulsory_bytes_per_image) (a per-op kernel: its input map + its output map, fp32, padded channel strides as
    stored; the stage: its input map, the taps and the head outputs) plus the regressors' tap reads
    and pose writes."""
    words = plan['words']
    flop = 0
    nbytes = 0
    off = int(words[BFH_OPS_OFF])
    staged = 0          # records left in the current stage: their maps stay in LDS
    fronted = 0         # records left in the front: only the frame and the last output touch HBM
    for i in range(int(words[BFH_NOPS])):
        f = [int(v) for v in words[off + i * BFO_WORDS: off + (i + 1) * BFO_WORDS]]
        if f[BFO_KIND] == BF_STAGE:
            staged = f[BFO_NI]
            first = True
            continue
        if f[BFO_KIND] == BF_FRONT:
            fronted = f[BFO_NI]
            continue
        if fronted:
            hw_in, hw_out = f[BFO_H] * f[BFO_W], f[BFO_HO] * f[BFO_WO]
            if f[BFO_KIND] == BF_STEM:
                flop += 2 * hw_out * 25 * 3 * f[BFO_COUT]
                nbytes += 4 * hw_in * 3
            else:
                flop += 2 * hw_out * 9 * f[BFO_CIN] + 2 * hw_out * f[BFO_CIN] * f[BFO_COUT]
                nbytes += 4 * hw_out * f[BFO_OSTRIDE] if fronted == 1 else 0
            fronted -= 1
            continue
        hw_in, hw_out = f[BFO_H] * f[BFO_W], f[BFO_HO] * f[BFO_WO]
        if f[BFO_KIND] == BF_STEM:
            flop += 2 * hw_out * 25 * 3 * f[BFO_COUT]
            nbytes += 4 * (hw_in * 3 + hw_out * f[BFO_COUTP])
            continue
        if f[BFO_DW]:
            flop += 2 * hw_out * 9 * f[BFO_CIN]
        flop += 2 * hw_out * f[BFO_CIN] * f[BFO_COUT]
        out_c = f[BFO_COUT] if f[BFO_SPLIT] else f[BFO_OSTRIDE]
        if staged:
            # inside a stage only the stage input, the taps and the head outputs touch HBM
            nbytes += 4 * (hw_in * f[BFO_CINP] if first else 0)
            nbytes += 4 * hw_out * out_c if f[BFO_DST] >= BUF_OUT0 else 0
            staged -= 1
            first = False
            continue
        nbytes += 4 * (hw_in * f[BFO_CINP] + hw_out * out_c)
    st = plan['structure']
    for r in st['regressors']:
        h, w, c = st['shapes'][r['tap']]
        layers = [l for l in r['config']['layers'] if l['class_name'] in ('Conv2D', 'Dense')]
        cin = c
        for l in layers:
            n = l['config'].get('filters', l['config'].get('units'))
            flop += 2 * h * w * cin * n
            cin = n
        nbytes += 4 * h * w * (c + 3)
    return flop, nbytes


def compulsory_bytes_per_image(plan):
    """Compulsory HBM bytes of one frame through the unified graph: the fp32
    input frame read once, and written once each: the four detector outputs, the two taps (the
    feature maps the caller keeps, hpe.features) and the two pose maps.  Everything else a
    forward moves (the 64x64 / 32x32 intermediate maps, the stage input, the taps' re-read by the
    pose heads) is plan traffic that a fully fused forward would not need (work_per_image)."""
    st = plan['structure']
    H, W = st['input_hw']
    n = 4 * H * W * 3
    heads = {hd['out']: hd['shape'] for hd in st['heads']}
    for o in plan['det_outs']:
        n += 4 * int(np.prod(heads[o]))
    for t in st['taps']:
        th, tw, c = st['shapes'][t]
        n += 4 * th * tw * c
    for r in st['regressors']:
        th, tw, _ = st['shapes'][r['tap']]
        n += 4 * th * tw * 3
    return n


class UnifiedModel:
    """Keras-model-shaped wrapper of a unified BlazeFace graph (what ``keras.models.load_model`` on
    ``BlazePoser/UnifiedModels/*.h5`` returns in the reference, blazeFaceDetectorH5.py:101):
    inference only — the reference never trains this graph."""

    def __init__(self, model_config, weights, name=None):
        self.model_config = model_config if 'config' in model_config else {'class_name': 'Functional',
                                                                            'config': model_config}
        self.name = name or self.model_config['config'].get('name', 'model')
        self._weights = dict(weights)
        self._bf = None
        parse(self.model_config)          # structure errors surface at load time (ValueError)

    def _net(self):
        if self._bf is None:
            self._bf = BlazeFace(self.model_config, self._weights)
        return self._bf

    def predict(self, x, batch_size=None, verbose=0, **kw):
        return self._net().predict(x)

    def __call__(self, x, training=False):
        if torch.is_tensor(x) and x.is_cuda:
            return self._net().forward(x)
        return self.predict(x)

    def count_params(self):
        return int(sum(np.asarray(v).size for v in self._weights.values()))

    def get_weights(self):
        return [np.asarray(v) for v in self._weights.values()]

    def weights_dict(self):
        return dict(self._weights)

    def to_json(self):
        import json
        return json.dumps(self.model_config)

    def compile(self, *a, **k):
        raise NotImplementedError('the unified BlazeFace graph is inference-only (as in the reference)')

    fit = compile
