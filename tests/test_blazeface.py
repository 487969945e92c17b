"""BlazeFace unified graph: structure recognition, plan packing (numpy
emulation of the plan words vs the oracle), the C-side plan validator (no GPU needed), and — on the
GPU — the fused HIP kernels against the oracle.

Parity is restatement-pinned (no TF output of the unified graph exists): the oracle
runs the unified model_config with Keras 2.13 layer semantics in float64.  Tolerance for the fp32
HIP path: rtol 1e-4, atol 1e-3 on every output (detector logits / box offsets in pixels / poses in
degrees; SURVEY.md allows 5e-2 deg for an fp16 path, this fp32 path is held 50x tighter)."""
import ctypes

import numpy as np
import pytest

import blaze_emu
from hpe import _lib
from hpe import blazeface as B
from oracle import keras_ref as K
from util import fixture

RID = 'reg1-stoqa9pt-reg2-hrchr82r-selected'
UNIFIED = [RID, 'reg1-stoqa9pt-reg2-cl4obelj', 'reg1-9w31h50k-reg2-cl4obelj', 'reg1-4121t6zb-reg2-cl4obelj']
BF_RTOL, BF_ATOL = 1e-4, 1e-3


def _images(n, seed=0):
    return np.random.default_rng(seed).uniform(-1, 1, (n, 128, 128, 3)).astype(np.float32)


def _oracle(n, seed=0):
    mc, w = fixture(RID)
    return [o.detach().numpy() for o in K.Graph(mc, w).forward(_images(n, seed))]


def test_structure_recognised():
    mc, _ = fixture(RID)
    st = B.parse(mc)
    assert len(st['blocks']) == 16
    assert [b['stride'] for b in st['blocks']].count(2) == 3
    assert [b['cout'] for b in st['blocks']][-1] == 96
    assert st['taps'] == ['re_lu_10', 're_lu_15']
    assert st['shapes']['re_lu_10'] == (16, 16, 88) and st['shapes']['re_lu_15'] == (8, 8, 96)
    assert [r['out'] for r in st['regressors']] == ['model', 'model_10']
    assert len(st["heads"]) == 4
    assert [h["shape"] for h in st["heads"]] == [(512, 1), (384, 1), (512, 16), (384, 16)]


def test_compulsory_bytes_per_frame():
    """bench.py's BlazeFace roofline counts each frame's compulsory HBM bytes:
    the 128x128x3 input, the 896-anchor detector outputs (1 score + 16 box values each), the two
    taps (16x16x88, 8x8x96) and the two 3-channel pose maps, fp32, once each."""
    mc, w = fixture(RID)
    plan = B.build_plan(mc, w)
    anchors = 16 * 16 * 2 + 8 * 8 * 6
    want = 4 * (128 * 128 * 3 + anchors * (1 + 16) + 16 * 16 * 88 + 8 * 8 * 96 + 16 * 16 * 3 + 8 * 8 * 3)
    assert B.compulsory_bytes_per_image(plan) == want == 376064
    # the per-op plan's traffic (every launch's input and output maps) is an order of magnitude
    # more; the front + stage plan keeps it within 2.5x (frame, front output, stage input / taps)
    assert B.work_per_image(B.build_plan(mc, w, stage=False, front=False))[1] > 10 * want
    assert B.work_per_image(plan)[1] < 2.5 * want


@pytest.mark.parametrize('rid', UNIFIED)
def test_plan_words_emulated_match_oracle(rid):
    mc, w = fixture(rid)
    plan = B.build_plan(mc, w)
    x = _images(2, seed=1)
    bufs = blaze_emu.run(plan, x)
    ref = K.Graph(mc, w).forward(x)
    for i, o in enumerate(plan['det_outs']):
        got = bufs[B.BUF_OUT0 + i].reshape(ref[i].shape)
        np.testing.assert_allclose(got, ref[i].detach().numpy(), rtol=1e-6, atol=1e-6, err_msg=o)
    g = K.Graph(mc, w)
    # taps against the oracle's intermediate activations (the regressors' inputs)
    for j, t in enumerate(plan['structure']['taps']):
        sub = dict(mc)
        cfg = dict(mc['config'])
        cfg['output_layers'] = [[t, 0, 0]]
        sub['config'] = cfg
        tap = K.Graph(sub, w).forward(x).detach().numpy()
        np.testing.assert_allclose(bufs[B.BUF_OUT0 + 4 + j], tap, rtol=1e-6, atol=1e-6, err_msg=t)
    del g


def test_rejects_unsupported_structure():
    mc, w = fixture(RID)
    import copy
    bad = copy.deepcopy(mc)
    for l in bad['config']['layers']:
        if l['name'] == 'depthwise_conv2d_3':
            l['config']['kernel_size'] = [5, 5]
    with pytest.raises(ValueError):
        B.parse(bad)


def test_capi_validates_plan_without_gpu():
    mc, w = fixture(RID)
    plan = B.build_plan(mc, w)
    lib = _lib.load()
    words = np.ascontiguousarray(plan['words'], np.int32)
    h = ctypes.c_void_p()
    assert lib.hpe_blazeface_create(words.ctypes.data_as(ctypes.c_void_p), words.size, ctypes.byref(h)) == 0
    assert lib.hpe_blazeface_workspace_size(h, 10) == 2 * 10 * int(words[B.BFH_ACT_FLOATS]) * 4
    assert lib.hpe_blazeface_destroy(h) == 0
    for field, val in ((B.BFO_LDS, 200_000), (B.BFO_NC, 7), (B.BFO_TH, 3), (B.BFO_SRC, 11)):
        bad = words.copy()
        bad[B.BFH_WORDS + 5 * B.BFO_WORDS + field] = val
        h2 = ctypes.c_void_p()
        assert lib.hpe_blazeface_create(bad.ctypes.data_as(ctypes.c_void_p), bad.size, ctypes.byref(h2)) == 1
    bad = words.copy()
    bad[0] = 0
    assert lib.hpe_blazeface_create(bad.ctypes.data_as(ctypes.c_void_p), bad.size, ctypes.byref(h)) == 1


def _records(words):
    off = int(words[B.BFH_OPS_OFF])
    return [[int(v) for v in words[off + i * B.BFO_WORDS: off + (i + 1) * B.BFO_WORDS]]
            for i in range(int(words[B.BFH_NOPS]))]


@pytest.mark.parametrize('rid', UNIFIED)
def test_stage_plan_covers_small_maps_and_heads(rid):
    """The plan's one BF_STAGE record covers every block from the 32x32 -> 16x16 stride-2 block on,
    each tap's two detector heads right after the block producing the tap; the per-op plan
    (stage=False) holds the same records in block-then-heads order."""
    mc, w = fixture(rid)
    recs = _records(B.build_plan(mc, w, front=False)['words'])
    per_op = _records(B.build_plan(mc, w, stage=False, front=False)['words'])
    k = [i for i, f in enumerate(recs) if f[B.BFO_KIND] == B.BF_STAGE]
    assert len(k) == 1
    st = recs[k[0]]
    covered = recs[k[0] + 1:k[0] + 1 + st[B.BFO_NI]]
    assert k[0] + 1 + st[B.BFO_NI] == len(recs)
    assert covered[0][B.BFO_HO] == 16 and covered[0][B.BFO_H] == 32 and covered[0][B.BFO_STRIDE] == 2
    assert all(f[B.BFO_HO] * f[B.BFO_WO] <= 256 for f in covered)
    assert sorted(map(tuple, covered)) == sorted(map(tuple, per_op[k[0]:]))
    for i, f in enumerate(covered):
        if not f[B.BFO_DW]:                       # heads read the tap the block before wrote
            prev = [g for g in covered[:i] if g[B.BFO_DW]][-1]
            assert f[B.BFO_SRC] == prev[B.BFO_DST] >= B.BUF_OUT0
    assert st[B.BFO_LDS] <= 160 * 1024
    assert B.work_per_image({'words': B.build_plan(mc, w)['words'], 'structure': B.parse(mc)})[0] == \
        B.work_per_image({'words': B.build_plan(mc, w, stage=False)['words'], 'structure': B.parse(mc)})[0]


@pytest.mark.parametrize('rid', UNIFIED)
def test_front_plan_covers_stem_and_large_maps(rid):
    """The plan's BF_FRONT record (bf_front_kernel) covers the stem and the five blocks on the
    64x64 / 32x32 maps, ahead of the stage; the records after it are the per-op plan's own, and
    the plan's HBM bytes drop to the frame, the front's 32x32x48 output and the stage's traffic."""
    mc, w = fixture(rid)
    recs = _records(B.build_plan(mc, w)['words'])
    per_op = _records(B.build_plan(mc, w, front=False)['words'])
    assert recs[0][B.BFO_KIND] == B.BF_FRONT and recs[0][B.BFO_NI] == 6
    assert recs[0][B.BFO_LDS] == B.FRONT_LDS <= 160 * 1024
    assert recs[1:] == per_op
    assert recs[1][B.BFO_KIND] == B.BF_STEM and recs[6][B.BFO_HO] == 32 and recs[7][B.BFO_KIND] == B.BF_STAGE
    plan, plan0 = B.build_plan(mc, w), B.build_plan(mc, w, front=False)
    f1, b1 = B.work_per_image(plan)
    f0, b0 = B.work_per_image(plan0)
    # the 64x64x24 (x4: stem out, block 1 in / out, block 2 in), 64x64x32 (x2), 32x32x32 (x2) and
    # 32x32x40 (x2) maps no longer touch HBM
    assert f1 == f0 and b0 - b1 == 4 * (4096 * 24 * 4 + 4096 * 32 * 2 + 1024 * 32 * 2 + 1024 * 40 * 2)


def test_capi_validates_front_record():
    mc, w = fixture(RID)
    words = np.ascontiguousarray(B.build_plan(mc, w)['words'], np.int32)
    lib = _lib.load()
    h = ctypes.c_void_p()
    assert lib.hpe_blazeface_create(words.ctypes.data_as(ctypes.c_void_p), words.size, ctypes.byref(h)) == 0
    lib.hpe_blazeface_destroy(h)
    base = B.BFH_WORDS
    for off, val in ((B.BFO_NI, 5), (B.BFO_LDS, 100_000), (B.BFO_WORDS + B.BFO_COUT, 16),
                     (3 * B.BFO_WORDS + B.BFO_COUTP, 40), (4 * B.BFO_WORDS + B.BFO_STRIDE, 1),
                     (6 * B.BFO_WORDS + B.BFO_DST, B.BUF_OUT0),
                     # an intermediate map the front keeps in LDS sent to a caller output
                     (1 * B.BFO_WORDS + B.BFO_DST, B.BUF_OUT0), (3 * B.BFO_WORDS + B.BFO_DST, B.BUF_OUT0 + 1),
                     # ... or read by the record after the front (block 4's map, never in HBM)
                     (8 * B.BFO_WORDS + B.BFO_SRC, int(words[base + 5 * B.BFO_WORDS + B.BFO_DST]))):
        bad = words.copy()
        bad[base + off] = val
        assert lib.hpe_blazeface_create(bad.ctypes.data_as(ctypes.c_void_p), bad.size, ctypes.byref(h)) == 1, off


def test_capi_validates_stage_record():
    mc, w = fixture(RID)
    words = np.ascontiguousarray(B.build_plan(mc, w, front=False)['words'], np.int32)
    recs = _records(words)
    k = [i for i, f in enumerate(recs) if f[B.BFO_KIND] == B.BF_STAGE][0]
    base = B.BFH_WORDS + k * B.BFO_WORDS
    lib = _lib.load()
    h = ctypes.c_void_p()
    assert lib.hpe_blazeface_create(words.ctypes.data_as(ctypes.c_void_p), words.size, ctypes.byref(h)) == 0
    lib.hpe_blazeface_destroy(h)
    for field, val in ((B.BFO_NI, 99), (B.BFO_NI, len(recs) - k), (B.BFO_LDS, 200_000), (B.BFO_CS, 64),
                       (B.BFO_ROWS, 100)):
        bad = words.copy()
        bad[base + field] = val
        assert lib.hpe_blazeface_create(bad.ctypes.data_as(ctypes.c_void_p), bad.size, ctypes.byref(h)) == 1, field
    # the first 8x8 head moved before the block that writes its tap
    bad = words.copy()
    a, b = base + 12 * B.BFO_WORDS, base + 13 * B.BFO_WORDS
    assert bad[b + B.BFO_DW] == 0
    bad[a:b + B.BFO_WORDS] = np.concatenate([words[b:b + B.BFO_WORDS], words[a:b]])
    assert lib.hpe_blazeface_create(bad.ctypes.data_as(ctypes.c_void_p), bad.size, ctypes.byref(h)) == 1


@pytest.mark.gpu
@pytest.mark.parametrize('rid', [RID, UNIFIED[2]])
def test_blazeface_stage_matches_per_op_bit_for_bit(rid):
    """bf_stage_kernel runs the same arithmetic as the per-op kernels (depthwise bias + 9 taps in
    order, fp16-split MFMA over ascending channel quads, bias, residual, ReLU): outputs and taps are
    bit-identical, at a ragged batch of 37 frames."""
    import torch
    mc, w = fixture(rid)
    x = torch.from_numpy(_images(37, seed=37)).cuda()
    res = {}
    for stage in (False, True):
        bf = B.BlazeFace(mc, w, stage=stage, front=False)
        outs = [o.cpu().numpy() for o in bf.forward(x)]
        res[stage] = (outs, {t: v.cpu().numpy() for t, v in bf.taps.items()})
    for o, a, b in zip(B.parse(mc)['outputs'], res[False][0], res[True][0]):
        np.testing.assert_array_equal(a, b, err_msg=o)
    for t in res[False][1]:
        np.testing.assert_array_equal(res[False][1][t], res[True][1][t], err_msg=t)


@pytest.mark.gpu
@pytest.mark.parametrize('rid,n', [(RID, 37), (UNIFIED[2], 5), (RID, 300)])
def test_blazeface_front_matches_per_op_bit_for_bit(rid, n):
    """bf_front_kernel (the stem and the five 64x64 / 32x32 blocks as one launch, maps streamed
    through LDS rings) runs the per-op kernels' arithmetic: with and without the stage behind it,
    every output and tap is bit-identical to the per-op plan; ragged batches, fewer frames than
    CUs (5) and more (300: workgroups walk several frames)."""
    import torch
    mc, w = fixture(rid)
    x = torch.from_numpy(_images(n, seed=n)).cuda()
    res = {}
    for front, stage in ((False, False), (True, False), (True, True)):
        bf = B.BlazeFace(mc, w, stage=stage, front=front)
        assert (B.BF_FRONT in [int(v) for v in bf.plan['words'][B.BFH_WORDS::B.BFO_WORDS]]) == front
        outs = [o.cpu().numpy() for o in bf.forward(x)]
        res[(front, stage)] = (outs, {t: v.cpu().numpy() for t, v in bf.taps.items()})
    ref = res[(False, False)]
    for key in ((True, False), (True, True)):
        for o, a, b in zip(B.parse(mc)['outputs'], ref[0], res[key][0]):
            np.testing.assert_array_equal(a, b, err_msg='%s %s' % (key, o))
        for t in ref[1]:
            np.testing.assert_array_equal(ref[1][t], res[key][1][t], err_msg='%s %s' % (key, t))


@pytest.mark.gpu
@pytest.mark.parametrize('rid,n', [(RID, 1), (RID, 5), (RID, 33)] + [(u, 3) for u in UNIFIED[1:]])
def test_blazeface_forward_matches_oracle(rid, n):
    mc, w = fixture(rid)
    bf = B.BlazeFace(mc, w)
    x = _images(n, seed=n)
    got = bf.predict(x)
    ref = [o.detach().numpy() for o in K.Graph(mc, w).forward(x)]
    for o, g, r in zip(bf.structure['outputs'], got, ref):
        assert g.shape == r.shape, (o, g.shape, r.shape)
        np.testing.assert_allclose(g, r, rtol=BF_RTOL, atol=BF_ATOL, err_msg=o)


@pytest.mark.gpu
def test_blazeface_batch_1024_sampled_oracle():
    """configs[4]'s batch (1,024 frames, blazeFaceDetectorH5.py:272): the persistent bf_direct /
    bf_rows grids run a different number of tasks per workgroup than at <= 33 frames.  Frames are
    independent, so 24 frames sampled across the batch (both ends, a stride through the middle)
    are checked against the oracle on those frames alone, and the whole batch against a second
    GPU run of the same frames in smaller batches (bit-identical: no cross-frame state)."""
    mc, w = fixture(RID)
    bf = B.BlazeFace(mc, w)
    x = _images(1024, seed=1024)
    got = bf.predict(x)
    pick = np.concatenate([np.arange(4), np.linspace(10, 1010, 16).astype(int), np.arange(1020, 1024)])
    ref = [o.detach().numpy() for o in K.Graph(mc, w).forward(x[pick])]
    for o, g, r in zip(bf.structure['outputs'], got, ref):
        np.testing.assert_allclose(g[pick], r, rtol=BF_RTOL, atol=BF_ATOL, err_msg=o)
    parts = [bf.predict(x[i:i + 100]) for i in range(0, 1024, 100)]
    for k, o in enumerate(bf.structure['outputs']):
        np.testing.assert_array_equal(got[k], np.concatenate([p[k] for p in parts]), err_msg=o)


@pytest.mark.gpu
def test_blazeface_taps_match_oracle():
    import torch
    mc, w = fixture(RID)
    bf = B.BlazeFace(mc, w)
    x = _images(3, seed=9)
    bf.forward(torch.from_numpy(x).cuda())
    for t, dev in bf.taps.items():
        cfg = dict(mc['config'])
        cfg['output_layers'] = [[t, 0, 0]]
        ref = K.Graph(dict(mc, config=cfg), w).forward(x).detach().numpy()
        np.testing.assert_allclose(dev.cpu().numpy(), ref, rtol=BF_RTOL, atol=BF_ATOL, err_msg=t)


def test_load_model_returns_unified_wrapper():
    import hpe
    from util import MODELS
    u = hpe.load_model(MODELS + '/' + RID)
    assert type(u).__name__ == 'UnifiedModel'
    assert u.count_params() == 101390 + 5891 + 3683       # backbone + stoqa9pt + hrchr82r
    with pytest.raises(NotImplementedError):
        u.compile(optimizer='adam')
