"""Attention heads on H x W > 1 maps (SURVEY.md §8 a9 SE, a10 spatial MHA; hpe/spatial.py).

CPU: the staged decomposition (SE gate -> program B -> attention core -> program D) emulated in
numpy (the row programs by the row-program emulator) against the oracle's forward of the
reference graph on 16x16 / 8x8 maps, for every SE + MHA checkpoint signature and for the
create_modelC (SE only) builder.  GPU: the HIP path (hpe_se_gate, hpe_mha, row programs) against
the oracle.  Parity source: oracle/keras_ref.py restates Keras GAP / MultiHeadAttention /
LayerNormalization (attention_model.py:34-72); no TF output exists for H x W > 1 (parity unpinned
beyond the restatement).
"""
import numpy as np
import pytest

import hpe.compiler as C
from hpe.spatial import SpatialPlan, is_spatial
import rowprog_emu as EMU
from oracle import keras_ref as K
from util import fixture, index

SPATIAL_IDS = [r for r in sorted(index()) if not r.startswith('reg1') and is_spatial(fixture(r)[0])]


def _flat(prog, w):
    p = np.zeros(prog.n_params)
    for k, (o, shp) in prog.param_index.items():
        p[o:o + int(np.prod(shp))] = w[k].ravel()
    p[prog.n_train:] = prog.consts
    return p


def _act(a, z):
    return EMU._act(a, z)


def _emulate(plan, x, P):
    """numpy restatement of the four stages (float64)."""
    n = x.shape[0] // P
    xg = x.astype(np.float64)
    if plan.pool:
        pd = C.compile_graph(plan.head_config, plan.head_weights, 'fwd', fused=False)
        rows = EMU.run(pd, _flat(pd, plan.head_weights), xg)['out']
        return rows.reshape(n, P, -1).mean(axis=1)
    if plan.se is not None:
        s = plan.se
        m = xg.reshape(n, P, -1).mean(axis=1)
        h = _act(s['act1'], m @ s['w1'] + s['b1'])
        g = _act(s['act2'], h @ s['w2'] + s['b2'])
        xg = (xg.reshape(n, P, -1) * g[:, None, :]).reshape(n * P, -1)
    if plan.mha is None:
        pd = C.compile_graph(plan.head_config, plan.head_weights, 'fwd', fused=False)
        return EMU.run(pd, _flat(pd, plan.head_weights), xg)['out']
    H, D = plan.mha['H'], plan.mha['D']
    pb = C.compile_graph(plan.qkv_config, plan.qkv_weights, 'fwd', fused=False)
    qkv = EMU.run(pb, _flat(pb, plan.qkv_weights), xg)['out']
    # program B: [q | k | v] rows (hpe_mha_xg takes xg from its own rows)
    q = qkv[:, :H * D].reshape(n, P, H, D)
    k = qkv[:, H * D:2 * H * D].reshape(n, P, H, D)
    v = qkv[:, 2 * H * D:].reshape(n, P, H, D)
    s = np.einsum('bthd,bshd->bhts', q, k)
    a = np.exp(s - s.max(-1, keepdims=True))
    a /= a.sum(-1, keepdims=True)
    o = np.einsum('bhts,bshd->bthd', a, v).reshape(n * P, H * D)
    pd = C.compile_graph(plan.head_config, plan.head_weights, 'fwd', fused=False)
    return EMU.run(pd, _flat(pd, plan.head_weights), np.concatenate([xg, o], axis=1))['out']


def _modelC():
    """attention_model.py:74-90 create_modelC (SE r=8 -> 11 units, 1x1-conv head), seeded weights."""
    from hpe import keras
    keras.backend.clear_session()
    inp = keras.Input((None, None, 88))
    se = keras.layers.GlobalAveragePooling2D()(inp)
    se = keras.layers.Dense(11, activation='relu')(se)
    se = keras.layers.Dense(88, activation='sigmoid')(se)
    se = keras.layers.Reshape((1, 1, 88))(se)
    x = keras.layers.Multiply()([inp, se])
    x = keras.layers.Conv2D(42, 1, activation='relu')(x)
    out = keras.layers.Conv2D(3, 1, activation=None)(x)
    m = keras.Model(inp, out)
    return m.model_config, m.weights_dict()


def assert_fp32_parity(got, ref, mc, w, x):
    """SURVEY §8(c)'s bound (rtol 1e-5, atol 1e-4), widened only where a plain fp32 evaluation of
    the same graph (the oracle in torch fp32, K.Graph(dtype=float32)) is itself further than that
    from the float64 oracle: atol = max(1e-4, 4 x that fp32 error).  The attention heads take a
    softmax over up to P = 2304 tokens of scores q.k whose fp32 rounding error grows with |q||k|
    and D (DESIGN.md §Oracle and parity), and LayerNorm divides by a small std afterwards, so the
    fp32 reference error is the honest floor, measured here rather than asserted."""
    import torch
    ref32 = K.Graph(mc, w, dtype=torch.float32).forward(x).detach().numpy()
    e32 = float(np.abs(ref32.astype(np.float64) - ref).max())
    atol = max(1e-4, 4.0 * e32)
    err = np.abs(got.astype(np.float64) - ref)
    bad = err > atol + 1e-5 * np.abs(ref)
    assert not bad.any(), ('max err %.3g (fp32 reference error %.3g, atol %.3g) at %d elements'
                           % (err.max(), e32, atol, int(bad.sum())))


def _inputs(n, h, w, c, seed):
    rng = np.random.default_rng(seed)
    return np.maximum(0.0, 0.6 * rng.standard_normal((n, h, w, c)) - 0.3).astype(np.float32)


def test_spatial_fixtures_present():
    assert len(SPATIAL_IDS) >= 5


@pytest.mark.parametrize('hw', [(16, 16), (8, 8)])
@pytest.mark.parametrize('rid', SPATIAL_IDS + ['create_modelC'])
def test_staged_decomposition_matches_oracle(rid, hw):
    mc, w = _modelC() if rid == 'create_modelC' else fixture(rid)
    c = mc['config']['layers'][0]['config']['batch_input_shape'][-1]
    x = _inputs(3, hw[0], hw[1], c, seed=sum(map(ord, rid)))
    ref = K.Graph(mc, w).forward(x).detach().numpy().reshape(-1, 3)
    plan = SpatialPlan(mc, w)
    got = _emulate(plan, x.reshape(-1, c), hw[0] * hw[1]).reshape(-1, 3)
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-5)


def _tail_weights(tail, C, HD):
    """Read the attention-tail buffer the way csrc/hpe_tail.hip does ([K/16][N/16][g][c][s] =
    W[16 bk + 4 g + s][16 bn + c]) back into plain [K][N] kernels and the vectors."""
    import hpe.spatial as S
    d, buf = tail['desc'], tail['w']
    FF, HID = int(d[S.TD_FF]), int(d[S.TD_HID])
    shapes = [(HD, C), (C, FF), (FF, C), (C, HID), (HID, 3)]
    out, off = [], 0
    for K_, N_ in shapes:
        kb, nb = -(-K_ // 16), -(-N_ // 16)
        blk = buf[off:off + kb * nb * 256].reshape(kb, nb, 4, 16, 4).transpose(0, 2, 4, 1, 3)
        out.append(blk.reshape(kb * 16, nb * 16)[:K_, :N_].astype(np.float64))
        off += kb * nb * 256
    assert off == int(d[S.TD_BO])
    sizes = [C, C, C, FF, C, C, C, HID, 3]
    vecs = [buf[int(d[S.TD_BO + i]):int(d[S.TD_BO + i]) + n].astype(np.float64) for i, n in enumerate(sizes)]
    return out, vecs, d


@pytest.mark.parametrize('rid', SPATIAL_IDS)
def test_attn_tail_plan_matches_oracle(rid):
    """The fused post-attention tail (csrc/hpe_tail.hip) as planned by hpe/spatial.py: its parameter
    buffer, read back in the kernel's MFMA operand order and evaluated in float64 after the staged
    SE gate / program B / attention core, reproduces the oracle's forward on 8x8 maps."""
    mc, w = fixture(rid)
    plan = SpatialPlan(mc, w)
    if plan.mha is None:
        pytest.skip('no attention core')
    assert plan.tail is not None, 'se_transformer_regr_head tail not recognised'
    c = plan.C
    H, D = plan.mha['H'], plan.mha['D']
    x = _inputs(2, 8, 8, c, seed=7)
    P = 64
    xr = x.reshape(-1, c).astype(np.float64)
    n = 2
    s = plan.se
    m = xr.reshape(n, P, -1).mean(axis=1)
    g = _act(s['act2'], _act(s['act1'], m @ s['w1'] + s['b1']) @ s['w2'] + s['b2'])
    xg = (xr.reshape(n, P, -1) * g[:, None, :]).reshape(n * P, -1)
    pb = C.compile_graph(plan.qkv_config, plan.qkv_weights, 'fwd', fused=False)
    qkv = EMU.run(pb, _flat(pb, plan.qkv_weights), xg)['out']
    q = qkv[:, :H * D].reshape(n, P, H, D)
    k = qkv[:, H * D:2 * H * D].reshape(n, P, H, D)
    v = qkv[:, 2 * H * D:].reshape(n, P, H, D)
    sc = np.einsum('bthd,bshd->bhts', q, k)
    a = np.exp(sc - sc.max(-1, keepdims=True))
    a /= a.sum(-1, keepdims=True)
    o = np.einsum('bhts,bshd->bthd', a, v).reshape(n * P, H * D)
    (wo, wf1, wf2, wc1, wc2), (bo, g1, be1, bf1, bf2, g2, be2, bc1, bc2), d = _tail_weights(plan.tail, c, H * D)
    import hpe.spatial as S

    def ln(t, gm, bt, eps):
        mu = t.mean(-1, keepdims=True)
        var = ((t - mu) ** 2).mean(-1, keepdims=True)
        return (t - mu) / np.sqrt(var + eps) * gm + bt
    eps1 = float(np.int32(d[S.TD_EPS1]).view(np.float32))
    eps2 = float(np.int32(d[S.TD_EPS2]).view(np.float32))
    t = ln(xg + o @ wo + bo, g1, be1, eps1)
    f = _act(int(d[S.TD_ACT_FF]), t @ wf1 + bf1) @ wf2 + bf2
    z = ln(t + f, g2, be2, eps2)
    y = _act(int(d[S.TD_ACT_OUT]), _act(int(d[S.TD_ACT_HID]), z @ wc1 + bc1) @ wc2 + bc2)
    ref = K.Graph(mc, w).forward(x).detach().numpy().reshape(-1, 3)
    np.testing.assert_allclose(y, ref, rtol=1e-5, atol=1e-5)


def test_row_local_graph_is_not_spatial():
    mc, w = fixture('hrchr82r')
    assert not is_spatial(mc)
    with pytest.raises(ValueError):
        SpatialPlan(mc, w)


# ------------------------------------------------------------------------------------------------
# GPU: the HIP path
# ------------------------------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize('hw', [(16, 16), (8, 8), (5, 7)])
@pytest.mark.parametrize('rid', SPATIAL_IDS + ['create_modelC'])
def test_gpu_spatial_predict_matches_oracle(rid, hw):
    import hpe
    mc, w = _modelC() if rid == 'create_modelC' else fixture(rid)
    c = mc['config']['layers'][0]['config']['batch_input_shape'][-1]
    x = _inputs(5, hw[0], hw[1], c, seed=7)
    ref = K.Graph(mc, w).forward(x).detach().numpy()
    m = hpe.model_from_config(mc, w)
    got = m.predict(x)
    assert got.shape == ref.shape
    assert_fp32_parity(got, ref, mc, w, x)


@pytest.mark.gpu
def test_gpu_spatial_large_map_and_p1_consistency():
    """48x48 maps (P = 2304 tokens: the attention streams 9 key blocks through LDS) on two images,
    and the P = 1 layout through the staged path equals the row program's."""
    import torch
    import hpe
    from hpe.spatial import SpatialHead
    rid = SPATIAL_IDS[0]
    mc, w = fixture(rid)
    c = mc['config']['layers'][0]['config']['batch_input_shape'][-1]
    x = _inputs(2, 48, 48, c, seed=3)
    ref = K.Graph(mc, w).forward(x).detach().numpy()
    got = hpe.model_from_config(mc, w).predict(x)
    assert_fp32_parity(got, ref, mc, w, x)
    x1 = _inputs(64, 1, 1, c, seed=4)
    m = hpe.model_from_config(mc, w)
    row = m.predict(x1).reshape(-1, 3)
    sh = SpatialHead(mc, w, torch.device('cuda'))
    staged = sh.forward(torch.from_numpy(x1.reshape(-1, c)).cuda(), 1).cpu().numpy()
    np.testing.assert_allclose(staged, row, rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize('D,P', [(16, 256), (6, 35), (48, 64)])
def test_mha_xg_matches_mha(D, P):
    """hpe_mha_xg (q | k | v rows + the pass-through columns from their own rows) against hpe_mha on
    the concatenated [xg | q | k | v] rows: identical outputs (same kernels, same arithmetic), for
    the MFMA core (key_dim <= 32) and the VALU one (key_dim 48)."""
    import ctypes
    import torch
    from hpe import _lib
    lib = _lib.load()
    n, C, H = 3, 88, 4
    g = torch.Generator().manual_seed(D + P)
    xg = torch.randn((n * P, C), generator=g).cuda()
    qkv = torch.randn((n * P, 3 * H * D), generator=g).cuda() * 0.5
    cat = torch.cat([xg, qkv], dim=1).contiguous()
    o1 = torch.zeros((n * P, C + H * D), device='cuda')
    o2 = torch.zeros_like(o1)
    vp = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert lib.hpe_mha(vp(cat), cat.shape[1], C, vp(o1), o1.shape[1], n, P, H, D, st) == 0
    assert lib.hpe_mha_xg(vp(qkv), qkv.shape[1], vp(xg), C, vp(o2), o2.shape[1], n, P, H, D, st) == 0
    torch.cuda.synchronize()
    assert torch.equal(o1, o2)
    assert torch.equal(o2[:, :C], xg)
