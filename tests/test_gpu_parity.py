"""GPU parity: the HIP path (libhpe.so through the C ABI) against the oracle on the reference's
own TF-trained checkpoints and datasets.  Forward tolerance rtol 1e-5 / atol 1e-4
degrees; MAE within 1e-4 degrees of the golden; training trajectories within the stated bounds."""
import os

import numpy as np
import pytest
import torch

import hpe
from hpe import keras
from oracle import keras_ref as K
from util import ATOL, RTOL, DATA, features, fixture, index, input_channels, labels

pytestmark = pytest.mark.gpu

FWD_IDS = sorted(r for r in index() if not r.startswith('reg1'))


@pytest.mark.parametrize('rid', FWD_IDS)
def test_forward_every_checkpoint_signature(rid):
    mc, w = fixture(rid)
    c = input_channels(mc)
    x = features(301, c, seed=len(rid))
    ref = K.Graph(mc, w).forward(x).detach().numpy().reshape(-1, 3)
    got = hpe.model_from_config(mc, w).predict(x).reshape(-1, 3)
    np.testing.assert_allclose(got, ref, rtol=RTOL, atol=ATOL)


GOLDEN_MAE = [  # BASELINE.md §2 (survey restatement of the reference's checkpoints on its data)
    ('stoqa9pt', 'AFLW2000_features_88_0.7_1.npz', 44.8263),
    ('stoqa9pt', 'AFLW2000_Enlarged_features_88_0.7_1.npz', 7.8100),
    ('stoqa9pt', 'BIWI_Test_Enlarged_features_88_0.7_1.npz', 3.4456),
    ('ker7z9mv', 'AFLW2000_Enlarged_features_88_0.7_1.npz', 7.9921),
    ('9w31h50k', 'AFLW2000_Enlarged_features_88_0.7_1.npz', 8.3447),
    ('hrchr82r', 'AFLW2000_features_96_0.7_1.npz', 8.0307),
    ('model_runid_hrchr82r', 'AFLW2000_features_96_0.7_1.npz', 8.0307),
    ('sqnu665j', 'AFLW2000_features_96_0.7_1.npz', 7.7826),
    ('o6e5xpan', 'AFLW2000_features_96_0.7_1.npz', 7.7222),
]


@pytest.mark.parametrize('rid,ds,golden', GOLDEN_MAE)
def test_golden_mae(rid, ds, golden):
    mc, w = fixture(rid)
    d = np.load(DATA + '/' + ds)
    x, y = d['features'], d['poses']
    m = hpe.model_from_config(mc, w)
    p = m.predict(x.reshape(-1, 1, 1, x.shape[1])).reshape(-1, 3)
    mae = np.mean(np.abs(p - y), axis=0)
    assert abs(float(np.mean(mae)) - golden) <= 1e-4 + 5e-5, (mae, golden)
    ref = K.Graph(mc, w).forward(x.reshape(-1, 1, 1, x.shape[1])).detach().numpy().reshape(-1, 3)
    np.testing.assert_allclose(p, ref, rtol=RTOL, atol=ATOL)


TRAIN_CASES = [
    ('sqnu665j', 'adam', 64, 3),      # create_model(360): 96-360 tanh-3
    ('0g73t16n', 'adam', 100, 2),     # create_model(256)
    ('hrchr82r', 'sgd', 128, 3),      # 96-32-16-3
    ('stoqa9pt', 'adam', 512, 2),     # 88-64 softsign-3, dropout 1e-4
    ('9w31h50k', 'adamax', 77, 2),    # create_model_complex: residual blocks
    ('ker7z9mv', 'adam', 50, 2),      # SE + MHA + LayerNorm head (P=1)
    ('o6e5xpan', 'sgd', 64, 2),       # SeparableConv2D
    # round 2: the 16 large signatures (generic interpreter beyond one launch's LDS / accumulators)
    ('3v3lb8ln', 'adam', 64, 2),      # create_model(512): 48 dW blocks, 12 waves
    ('8equl7wt', 'sgd', 100, 2),      # 512-256-128-3: 208 dW blocks -> 2 passes per step
    ('66kjr5zw', 'adam', 100, 2),     # 512-256-128 residual + dropout: 3 passes, slots in device scratch
    ('6togj6se', 'adamax', 77, 2),    # 11-layer residual tanh stack: slots in device scratch
    ('s25l3n04', 'adam', 128, 2),     # 512-256-256-... residual: 3 passes + device-scratch slots
    # 128-wide residual relu stack with Activation layers and dropout.  With round 4's dropout masks
    # the trajectory is ill-conditioned at fp32 resolution: the oracle run in torch fp32 moves one
    # conv2d_2/kernel element 4.2e-5 from float64 (the HIP path: 3.9e-5); the test widens the bar to
    # the measured fp32 floor for such elements only
    ('rtomubjl', 'adamax', 64, 2),
    ('rd93oeou', 'adam', 100, 2),     # 256-128-... residual tanh stack: device-scratch slots
    ('rkq8scme', 'sgd', 90, 2),       # residual stack ending 32-8-3
    ('rdsncwuy', 'adamax', 128, 2),   # 128-256-512-3 with dropout: 2 passes
    ('jgbwpv9i', 'adam', 100, 2),     # 512-256-128 residual (no dropout): 3 passes + device slots
    # create_model(350), dropout 0.01, the fused 12-wave kernel.  SGD: under Adam, weights whose
    # gradient is near zero (data term cancelling the L2 term) take a +-lr step whose sign is set by
    # rounding (m / sqrt(v) ~ sign(g)), so no fp32 run tracks the float64 oracle there
    ('i1tlps36', 'sgd', 128, 2),
    ('08xjpkmi', 'sgd', 64, 2),       # create_model(360) variant
]


def _oracle_fit(mc, w, opt, x, y, bs, epochs, dtype=None):
    g = K.Graph(mc, w) if dtype is None else K.Graph(mc, w, dtype=dtype)
    o = K.LegacyOptimizer(opt, 2.8e-4 if opt != 'sgd' else 0.05)
    n = x.shape[0]
    it = 0
    for _ in range(epochs):               # shuffle=False: batches in order, last one partial
        for b0 in range(0, n, bs):
            it += 1
            K.train_step(g, o, x[b0:b0 + bs], y[b0:b0 + bs], drop_seed=hpe.random.dropout_seed(it))
    return g


@pytest.mark.parametrize('rid,opt,bs,epochs', TRAIN_CASES)
def test_training_trajectory(rid, opt, bs, epochs):
    mc, w = fixture(rid)
    c = input_channels(mc)
    n = 200
    x = features(n, c, seed=3)
    y = labels(n, seed=4)
    hpe.set_seed(7)
    m = hpe.model_from_config(mc, w)
    lr = 2.8e-4 if opt != 'sgd' else 0.05
    m.compile(optimizer={'adam': keras.optimizers.Adam, 'sgd': keras.optimizers.SGD,
                         'adamax': keras.optimizers.Adamax}[opt](learning_rate=lr),
              loss='mse', metrics=['mae'])
    hist = m.fit(x, y, batch_size=bs, epochs=epochs, shuffle=False, verbose=0)
    g = _oracle_fit(mc, w, opt, x, y, bs, epochs)
    got = m.weights_dict()
    bad = [k for k in g.trainable
           if not np.allclose(got[k], g.params[k].detach().numpy(), rtol=2e-4, atol=2e-5)]
    if bad:
        # fp32 conditioning floor of this trajectory: the same oracle evaluated in fp32 (torch CPU).
        # An element whose update is set by a rounding-level quantity (Adam / Adamax on a
        # near-zero gradient, a unit at a relu kink) moves by up to an lr-sized step under ANY fp32
        # evaluation; such an element may deviate from float64 by twice what the fp32 oracle itself
        # deviates, every other element keeps the 2e-4 / 2e-5 bar
        g32 = _oracle_fit(mc, w, opt, x, y, bs, epochs, dtype=torch.float32)
        for k in bad:
            ref = g.params[k].detach().numpy().astype(np.float64)
            floor = np.abs(g32.params[k].detach().numpy().astype(np.float64) - ref)
            err = np.abs(got[k].astype(np.float64) - ref)
            tol = 2e-5 + 2e-4 * np.abs(ref) + 2.0 * floor
            print('%s %s: %d elements past the bar, fp32 oracle floor max %.2e, HIP max err %.2e'
                  % (rid, k, int((err > 2e-5 + 2e-4 * np.abs(ref)).sum()), floor.max(), err.max()))
            assert (err <= tol).all(), (k, float(err.max()), float(floor.max()))
    pr = m.predict(x).reshape(-1, 3)
    pref = g.forward(x).detach().numpy().reshape(-1, 3)
    np.testing.assert_allclose(pr, pref, rtol=1e-4, atol=1e-3)
    assert np.isfinite(hist.history['loss']).all()


def test_spatial_forward_96x96():
    """Fully-convolutional head on a literal 96x96 map (P = 9216 rows per image)."""
    mc, w = fixture('hrchr82r')
    x = features(2, 96, seed=5, h=96, w=96)
    ref = K.Graph(mc, w).forward(x).detach().numpy()
    got = hpe.model_from_config(mc, w).predict(x)
    assert got.shape == (2, 96, 96, 3)
    np.testing.assert_allclose(got, ref, rtol=RTOL, atol=ATOL)


def test_spatial_train_step_grad():
    """One training step at P = 16x16 against autodiff (labels broadcast over H, W)."""
    mc, w = fixture('sqnu665j')
    x = features(6, 96, seed=6, h=16, w=16)
    y = labels(6, seed=7)
    m = hpe.model_from_config(mc, w)
    m.compile(optimizer=keras.optimizers.SGD(learning_rate=0.5), loss='mse', metrics=['mae'])
    m.fit(x, y, batch_size=6, epochs=1, shuffle=False, verbose=0)
    g = K.Graph(mc, w)
    K.train_step(g, K.LegacyOptimizer('sgd', 0.5), x, y, drop_seed=hpe.random.dropout_seed(1))
    got = m.weights_dict()
    for k in g.trainable:
        np.testing.assert_allclose(got[k], g.params[k].numpy(), rtol=1e-4, atol=1e-5, err_msg=k)


def test_evaluate_matches_oracle():
    mc, w = fixture('stoqa9pt')
    d = np.load(DATA + '/AFLW2000_Enlarged_features_88_0.7_1.npz')
    x, y = d['features'].reshape(-1, 1, 1, 88), d['poses']
    m = hpe.model_from_config(mc, w)
    m.compile(optimizer=keras.optimizers.SGD(learning_rate=2.8e-4), loss='mse', metrics=['mae'])
    loss, mae = m.evaluate(x, y.reshape(-1, 1, 1, 3))
    g = K.Graph(mc, w)
    p = g.forward(x).detach().numpy().reshape(-1, 3)
    ref_mse = float(np.mean((p - y) ** 2)) + float(g.regularization().item())
    assert abs(loss - ref_mse) <= 1e-4 * ref_mse
    assert abs(mae - float(np.mean(np.abs(p - y)))) <= 1e-4


@pytest.mark.parametrize('rid', ['hrchr82r', 'fsjbki8r', '0klags84'])
def test_chain_forward_ragged_and_gather(rid):
    """Fused chain forward (csrc/hpe_chain.hip): ragged tails (n % 32 != 0), several tiles per wave
    (n >> 32 x 12 waves x 256 CUs) and the image-index gather at P = 1 and P = 4."""
    from hpe.engine import Engine
    mc, w = fixture(rid)
    c = input_channels(mc)
    eng = Engine(mc, w)
    assert eng.program('fwd', 1).prog.kind == 'chain'
    g = K.Graph(mc, w)
    for n in (1, 31, 33, 385, 100_003, 400_001):
        x = features(n, c, seed=n)
        ref = g.forward(x).detach().numpy().reshape(-1, 3)
        got = eng.forward(torch.from_numpy(x.reshape(n, c)).cuda(), 1).cpu().numpy()
        np.testing.assert_allclose(got, ref, rtol=RTOL, atol=ATOL, err_msg='n=%d' % n)
    flat = any(l['class_name'] == 'Flatten' for l in mc['config']['layers'])
    for P in ((1,) if flat else (1, 4)):     # Flatten heads are row-local only at P == 1
        n_img = 777
        x = features(n_img, c, seed=P, h=1, w=P)
        idx = np.random.default_rng(P).permutation(n_img)[:301].astype(np.int32)
        ref = g.forward(x[idx]).detach().numpy().reshape(-1, 3)
        got = eng.forward(torch.from_numpy(x.reshape(-1, c)).cuda(), P,
                          idx=torch.from_numpy(idx).cuda()).cpu().numpy()
        np.testing.assert_allclose(got, ref, rtol=RTOL, atol=ATOL, err_msg='P=%d' % P)


def test_chain_split_precision_and_overflow_guard():
    """The chain kernel runs its GEMMs as fp16 hi/lo splits (csrc/hpe_common.h mfma3): its error
    against the float64 oracle stays at the exact-fp32 kernel's level, and inputs outside the fp16
    range (a feature >= 65504) are recomputed by the exact-fp32 twin (guard word), not mangled."""
    from hpe import _lib
    from hpe.engine import Engine
    mc, w = fixture('hrchr82r')
    eng = Engine(mc, w)
    g = K.Graph(mc, w)
    n = 100_003
    x = features(n, 96, seed=11)
    ref = g.forward(x).detach().numpy().reshape(-1, 3)
    xt = torch.from_numpy(x.reshape(n, 96)).cuda()
    lib = _lib.load()
    prev = lib.hpe_set_exact_fp32(1)
    try:
        exact = eng.forward(xt, 1).cpu().numpy()
    finally:
        lib.hpe_set_exact_fp32(prev)
    split = eng.forward(xt, 1).cpu().numpy()
    e_exact = float(np.abs(exact - ref).max())
    e_split = float(np.abs(split - ref).max())
    print('max |err| vs float64 oracle: exact fp32 %.3e, fp16-split %.3e' % (e_exact, e_split))
    assert e_split <= 4 * e_exact + 2e-6, (e_split, e_exact)
    np.testing.assert_allclose(split, ref, rtol=RTOL, atol=ATOL)
    xo = x.reshape(n, 96).copy()
    xo[5, 3] = 1.0e5
    xo[70_000, 10] = -7.0e4
    refo = g.forward(xo.reshape(n, 1, 1, 96)).detach().numpy().reshape(-1, 3)
    got = eng.forward(torch.from_numpy(xo).cuda(), 1).cpu().numpy()
    assert np.isfinite(got).all()
    np.testing.assert_allclose(got, refo, rtol=RTOL, atol=ATOL)
    # the next launch (new epoch) is back on the split path and still right
    np.testing.assert_allclose(eng.forward(xt, 1).cpu().numpy(), ref, rtol=RTOL, atol=ATOL)


def _data_grad64(mc, w, x, y, layout, seed):
    """float64 oracle gradient of the data term (mse) in the engine's flat parameter order."""
    g = K.Graph(mc, w)
    tr = list(g.trainable)
    for k in tr:
        g.params[k].requires_grad_(True)
    p = g.forward(x, training=True, drop_seed=seed)
    yt = torch.tensor(np.asarray(y), dtype=torch.float64)
    yb = yt.reshape(yt.shape[0], *([1] * (p.dim() - 2)), 3).expand_as(p)
    gr = torch.autograd.grad(K.mse(yb, p), [g.params[k] for k in tr])
    flat = np.zeros(sum(int(np.prod(s)) for _, s in layout.param_index.values()))
    for k, gk in zip(tr, gr):
        o, shp = layout.param_index[k]
        flat[o:o + int(np.prod(shp))] = gk.detach().numpy().ravel()
    return flat


@pytest.mark.parametrize('rid,P', [('sqnu665j', 1), ('sqnu665j', 96 * 96), ('stoqa9pt', 4 * 4)])
def test_train_step_split_vs_exact_and_guard(rid, P):
    """The fused training step's exponent-shifted fp16-split GEMMs (csrc/hpe_mlp2.hip SPLIT,
    hpe_common.h split_w8 / split_d8) against its exact-fp32 instantiation and the float64 oracle,
    with the reference's trained weights (sqnu665j: create_model(360), l2 0.1, 28 % of |W1| < 6e-5;
    stoqa9pt: 88-64-3 on 4x4 maps — at P = 1 it trains on the exact-fp32 wide kernel of
    csrc/hpe_res.hip) at P = 1 and on 96x96 maps.  Bars: the split gradient's error against
    float64 (normwise, max |err| / max |g|) within 4x the exact-fp32 kernel's own, and split vs
    exact within 1e-6 of max |g|.  A feature outside the fp16 range of the data side (|x| >= 64)
    makes the split launch hand the step to the exact one (guard word)."""
    from hpe import _lib
    from hpe.engine import Engine
    mc, w = fixture(rid)
    c = input_channels(mc)
    eng = Engine(mc, w)
    assert eng.program('train', P).prog.kind == 'mlp2'
    n = 3000 if P == 1 else (200 if P <= 64 else 2)
    side = int(round(P ** 0.5))
    x = features(n, c, seed=21, h=side, w=side)
    y = labels(n, seed=22)
    xt = torch.from_numpy(x.reshape(n * P, c)).cuda()
    yt = torch.from_numpy(y.reshape(n, 3).astype(np.float32)).cuda()
    inv = 1.0 / (n * P * 3)

    def grad(xd):
        return eng.gradient(xd, yt, P, None, n, inv, seed=5).cpu().numpy().copy()

    lib = _lib.load()
    prev = lib.hpe_set_exact_fp32(1)
    try:
        g_exact = grad(xt)
    finally:
        lib.hpe_set_exact_fp32(prev)
    g_split = grad(xt)
    npt = eng.n_train
    g64 = _data_grad64(mc, w, x, y, eng.layout, 5)
    scale = np.abs(g64).max()
    e_exact = np.abs(g_exact[:npt] - g64).max() / scale
    e_split = np.abs(g_split[:npt] - g64).max() / scale
    d = np.abs(g_split[:npt] - g_exact[:npt]).max() / scale
    print('%s P=%d: vs float64 exact %.2e split %.2e; |split - exact| / max|g| = %.2e' % (rid, P, e_exact, e_split, d))
    assert e_split <= 4 * e_exact + 2.0 ** -24, (e_split, e_exact)
    assert d <= 1e-6, d
    np.testing.assert_allclose(g_split[npt:npt + 2], g_exact[npt:npt + 2], rtol=1e-5)
    # guard: one feature at 100 (beyond the data side's 64) -> the split launch flags, the exact
    # instantiation recomputes
    xo = x.reshape(n * P, c).copy()
    xo[17, 5] = 100.0
    xot = torch.from_numpy(xo).cuda()
    prev = lib.hpe_set_exact_fp32(1)
    try:
        go_exact = grad(xot)
    finally:
        lib.hpe_set_exact_fp32(prev)
    go = grad(xot)
    assert np.isfinite(go).all()
    np.testing.assert_array_equal(go, go_exact)


@pytest.mark.parametrize('rid,P,n', [('sqnu665j', 1, 128), ('stoqa9pt', 1, 500), ('sqnu665j', 64, 4)])
def test_train_step_bounded_matches_unbounded(rid, P, n):
    """hpe_train_step_bounded (fit's per-step launches: x_bound = max |x| of the resident rows,
    below the fp16 split's data range) launches no exact-fp32 twin; the split kernel's result is
    the same bits as the guarded launch's (the twin exits without writing when the guard is clear)."""
    from hpe.engine import Engine
    mc, w = fixture(rid)
    c = input_channels(mc)
    eng = Engine(mc, w)
    side = int(round(P ** 0.5))
    x = features(n, c, seed=31, h=side, w=side)
    y = labels(n, seed=32)
    xt = torch.from_numpy(x.reshape(n * P, c)).cuda()
    yt = torch.from_numpy(y.reshape(n, 3).astype(np.float32)).cuda()
    bound = float(np.abs(x).max())
    assert 0 < bound < 64
    g0 = eng.gradient(xt, yt, P, None, n, 1.0 / (n * P * 3), seed=3).cpu().numpy().copy()
    g1 = eng.gradient(xt, yt, P, None, n, 1.0 / (n * P * 3), seed=3, x_bound=bound).cpu().numpy().copy()
    np.testing.assert_array_equal(g0, g1)


@pytest.mark.parametrize('F,act,dropout,side,n', [(360, 'tanh', 0.0, 96, 2), (360, 'tanh', 0.3, 8, 300),
                                                  (200, 'elu', 0.2, 6, 500), (256, 'relu', 0.1, 12, 120),
                                                  (137, 'softsign', 0.0, 33, 16), (360, 'tanh', 0.3, 8, 40)])
def test_train_step_12wave_kernel(F, act, dropout, side, n):
    """The fused split training step of the 12-wave mlp2_kernel (csrc/hpe_mlp2.hip) at P >= 32,
    128 < F <= 384 (the configs[3] shape and its neighbours).  Checks the
    gradient (incl. loss sums) against the exact-fp32 12-wave kernel and the float64 oracle,
    for the compiled-in tanh / softsign, the runtime-activation instantiation (elu, relu) and
    SpatialDropout on both layers; ragged row counts (n P not a multiple of the 32-row tile)."""
    from hpe import _lib
    hpe.set_seed(F)
    m = _create_model(F, act, dropout, 0.1)
    mc, w = m.model_config, m.weights_dict()
    eng = m._eng()
    P = side * side
    assert eng.program('train', P).prog.kind == 'mlp2'
    x = features(n, 96, seed=F + 7, h=side, w=side)
    y = labels(n, seed=F + 8)
    xt = torch.from_numpy(x.reshape(n * P, 96)).cuda()
    yt = torch.from_numpy(y.reshape(n, 3).astype(np.float32)).cuda()
    inv = 1.0 / (n * P * 3)

    def grad():
        return eng.gradient(xt, yt, P, None, n, inv, seed=5).cpu().numpy().copy()

    lib = _lib.load()
    prev = lib.hpe_set_exact_fp32(1)
    try:
        g_exact = grad()
    finally:
        lib.hpe_set_exact_fp32(prev)
    g_split = grad()
    npt = eng.n_train
    g64 = _data_grad64(mc, w, x, y, eng.layout, 5)
    scale = np.abs(g64).max()
    e_exact = np.abs(g_exact[:npt] - g64).max() / scale
    e_split = np.abs(g_split[:npt] - g64).max() / scale
    d = np.abs(g_split[:npt] - g_exact[:npt]).max() / scale
    print('F=%d %s drop %.2f P=%d: vs float64 exact %.2e split %.2e; |split - exact| / max|g| = %.2e'
          % (F, act, dropout, P, e_exact, e_split, d))
    assert e_split <= 4 * e_exact + 2.0 ** -24, (e_split, e_exact)
    assert d <= 1e-6, d
    np.testing.assert_allclose(g_split[npt:npt + 2], g_exact[npt:npt + 2], rtol=1e-5)


@pytest.mark.parametrize('rid,side,n,R', [('sqnu665j', 96, 2, 60), ('sqnu665j', 96, 24, 12),
                                          ('stoqa9pt', 88, 8, 24),
                                          # one tile per workgroup (8 tiles on 8 workgroups / 40 tiles)
                                          ('sqnu665j', 8, 4, 40), ('sqnu665j', 8, 40, 40),
                                          (('tanh', 0.3), 8, 4, 40), (('tanh', 0.3), 8, 40, 40)])
def test_train_step_repeatable(rid, side, n, R):
    """Race screen (scripts/diag_repeat.py as a test): the fused training step launched R times on
    identical inputs must give bit-identical gradients.  sqnu665j at 96x96 runs the split 12-wave
    kernel (n = 2: two or three tiles per workgroup, the first tile's X(t+1) staged right before
    forward(0); n = 24: the steady-state staging), stoqa9pt at 88x88 the 4-wave mlp2_kernel.  The
    8x8 cases launch one 32-row tile per workgroup (the launch shape where round 4's 8-wave kernel
    dropped dW2 row terms), without and with SpatialDropout on both layers (create_model(360, tanh,
    0.3)), including a process's first launches."""
    from hpe.engine import Engine
    if isinstance(rid, tuple):
        hpe.set_seed(360)
        m = _create_model(360, rid[0], rid[1], 0.1)
        eng, c = m._eng(), 96
    else:
        mc, w = fixture(rid)
        c = input_channels(mc)
        eng = Engine(mc, w)
    P = side * side
    assert eng.program('train', P).prog.kind == 'mlp2'
    x = features(n, c, seed=21, h=side, w=side)
    y = labels(n, seed=22)
    xt = torch.from_numpy(x.reshape(n * P, c)).cuda()
    yt = torch.from_numpy(y.reshape(n, 3).astype(np.float32)).cuda()
    inv = 1.0 / (n * P * 3)
    ref = eng.gradient(xt, yt, P, None, n, inv, seed=5).cpu().numpy().copy()
    assert np.isfinite(ref).all()
    for r in range(1, R):
        g = eng.gradient(xt, yt, P, None, n, inv, seed=5).cpu().numpy()
        assert np.array_equal(g, ref), 'run %d differs from run 0 in %d entries' % (r, int((g != ref).sum()))


@pytest.mark.parametrize('F,act,dropout,cin,side,n', [(64, 'softsign', 0.2, 88, 88, 8), (64, 'tanh', 0.0, 96, 87, 5),
                                                      (40, 'softsign', 0.3, 88, 64, 10), (64, 'softsign', 1e-4, 88, 88, 6),
                                                      (64, 'softsign', 0.1, 88, 87, 5)])
def test_train_step_rows_kernel(F, act, dropout, cin, side, n):
    """The row-parallel split training kernel for narrow hidden layers (csrc/hpe_mlp2.hip
    mlp2r_kernel: F <= 64, launches of >= 2^15 rows, train_88.py:66-140's 88 -> 64 softsign -> 3)
    against the exact-fp32 kernel and the float64 oracle (same bars as the 12-wave kernel's test),
    against the unit-split kernel it replaces (HPE_MLP2_ROWS=0: same products, another summation
    order), ragged rows (87 x 87 maps), F < 64, dropout on both layers; then the guard: a feature
    beyond the split's data range hands the launch to the exact twin."""
    from hpe import _lib
    hpe.set_seed(F + cin)
    keras.backend.clear_session()
    reg = keras.regularizers.l2(1e-6)
    inp = keras.Input(shape=(None, None, cin))
    h = keras.layers.Conv2D(F, 1, padding='same', activation=act, kernel_regularizer=reg)(inp)
    h = keras.layers.SpatialDropout2D(dropout)(h)
    o = keras.layers.Conv2D(3, 1, padding='same', kernel_regularizer=reg)(h)
    o = keras.layers.SpatialDropout2D(dropout)(o)
    m = keras.Model(inp, o)
    m.compile(optimizer=keras.optimizers.Adam(learning_rate=2.8e-4), loss='mse', metrics=['mae'])
    mc, w = m.model_config, m.weights_dict()
    eng = m._eng()
    P = side * side
    assert eng.program('train', P).prog.kind == 'mlp2' and n * P >= 1 << 15
    x = features(n, cin, seed=F + 3, h=side, w=side)
    y = labels(n, seed=F + 4)
    xt = torch.from_numpy(x.reshape(n * P, cin)).cuda()
    yt = torch.from_numpy(y.reshape(n, 3).astype(np.float32)).cuda()
    inv = 1.0 / (n * P * 3)

    def grad(xd):
        return eng.gradient(xd, yt, P, None, n, inv, seed=5).cpu().numpy().copy()

    lib = _lib.load()
    prev = lib.hpe_set_exact_fp32(1)
    try:
        g_exact = grad(xt)
    finally:
        lib.hpe_set_exact_fp32(prev)
    g_rows = grad(xt)
    os.environ['HPE_MLP2_ROWS'] = '0'
    try:
        g_units = grad(xt)
    finally:
        del os.environ['HPE_MLP2_ROWS']
    assert not np.array_equal(g_rows, g_units)  # the two kernels ran (different summation orders)
    npt = eng.n_train
    g64 = _data_grad64(mc, w, x, y, eng.layout, 5)
    scale = np.abs(g64).max()
    e_exact = np.abs(g_exact[:npt] - g64).max() / scale
    e_rows = np.abs(g_rows[:npt] - g64).max() / scale
    e_units = np.abs(g_units[:npt] - g64).max() / scale
    d = np.abs(g_rows[:npt] - g_exact[:npt]).max() / scale
    print('F=%d %s drop %g cin %d P=%d: vs float64 exact %.2e rows %.2e units %.2e; |rows - exact| / max|g| = %.2e'
          % (F, act, dropout, cin, P, e_exact, e_rows, e_units, d))
    assert e_rows <= 4 * e_exact + 2.0 ** -24, (e_rows, e_exact)
    assert d <= 1e-6, d
    np.testing.assert_allclose(g_rows[npt:npt + 2], g_exact[npt:npt + 2], rtol=1e-5)
    np.testing.assert_allclose(g_rows[npt:npt + 2], g_units[npt:npt + 2], rtol=1e-5)
    xo = x.reshape(n * P, cin).copy()
    xo[(n * P) // 2 + 1, 7] = 100.0
    xot = torch.from_numpy(xo).cuda()
    prev = lib.hpe_set_exact_fp32(1)
    try:
        go_exact = grad(xot)
    finally:
        lib.hpe_set_exact_fp32(prev)
    go = grad(xot)
    assert np.isfinite(go).all()
    np.testing.assert_array_equal(go, go_exact)


def test_rows_kernel_fit_matches_oracle():
    """Model.fit on mlp2r_kernel (F = 64 softsign, dropout on both layers, 88x88 maps: 8 images =
    61,952 rows per step) through fit's gathered batches (the image-index LDS-DMA path of the packed
    88-float rows), 2 epochs of Adam against the oracle's fit with the same dropout masks."""
    hpe.set_seed(5)
    keras.backend.clear_session()
    reg = keras.regularizers.l2(1e-6)
    inp = keras.Input(shape=(None, None, 88))
    h = keras.layers.Conv2D(64, 1, padding='same', activation='softsign', kernel_regularizer=reg)(inp)
    h = keras.layers.SpatialDropout2D(0.1)(h)
    o = keras.layers.Conv2D(3, 1, padding='same', kernel_regularizer=reg)(h)
    o = keras.layers.SpatialDropout2D(0.1)(o)
    m = keras.Model(inp, o)
    m.compile(optimizer=keras.optimizers.Adam(learning_rate=2.8e-4), loss='mse', metrics=['mae'])
    w0 = m.weights_dict()
    n, side, bs = 12, 88, 8
    x = features(n, 88, seed=9, h=side, w=side)
    y = labels(n, seed=10)
    hist = m.fit(x, y, batch_size=bs, epochs=2, shuffle=False, verbose=0)
    g = _oracle_fit(m.model_config, w0, 'adam', x, y, bs, 2)
    got = m.weights_dict()
    for k in g.trainable:
        np.testing.assert_allclose(got[k], g.params[k].detach().numpy(), rtol=2e-4, atol=2e-5, err_msg=k)
    assert np.isfinite(hist.history['loss']).all()


def _create_model(F, act, dropout, l2, lr=2.8e-4):
    """train_96.py:65-110 create_model with the given width / activation / rates."""
    keras.backend.clear_session()
    reg = keras.regularizers.l2(l2)
    inp = keras.Input(shape=(None, None, 96))
    h = keras.layers.Conv2D(F, 1, padding='same', activation=act, kernel_regularizer=reg,
                            bias_regularizer=reg)(inp)
    h = keras.layers.SpatialDropout2D(dropout)(h)
    o = keras.layers.Conv2D(3, 1, padding='same', kernel_regularizer=reg, bias_regularizer=reg)(h)
    o = keras.layers.SpatialDropout2D(dropout)(o)
    m = keras.Model(inp, o)
    m.compile(optimizer=keras.optimizers.Adam(learning_rate=lr), loss='mse', metrics=['mae'])
    return m


@pytest.mark.parametrize('F,act,dropout,P', [(360, 'tanh', 0.05, 1), (360, 'tanh', 0.3, 16),
                                             (256, 'relu', 0.1, 1), (200, 'elu', 0.2, 4),
                                             (360, 'tanh', 0.3, 64), (200, 'elu', 0.2, 36)])
def test_training_trajectory_wide_dropout(F, act, dropout, P):
    """the 12-wave split kernel (129 <= F <= 384) with dropout on both layers (the
    sweep.yaml grid: filters 256 / 360, dropout > 0), for the compiled-in tanh and the runtime
    activation instantiation (ACT1 = -1), against the oracle's fit with the same dropout masks;
    at P >= 32 fit's gathered batches run the split 12-wave kernel."""
    hpe.set_seed(11)
    m = _create_model(F, act, dropout, 0.1)
    w0 = m.weights_dict()
    assert m._eng().program('train', P).prog.info.get('waves') == -(-F // 32)
    side = int(round(P ** 0.5))
    n = 120 if P == 1 else 24
    x = features(n, 96, seed=F, h=side, w=side)
    y = labels(n, seed=F + 1)
    hist = m.fit(x, y, batch_size=40 if P == 1 else 8, epochs=2, shuffle=False, verbose=0)
    g = _oracle_fit(m.model_config, w0, 'adam', x, y, 40 if P == 1 else 8, 2)
    got = m.weights_dict()
    for k in g.trainable:
        np.testing.assert_allclose(got[k], g.params[k].detach().numpy(), rtol=2e-4, atol=2e-5, err_msg=k)
    assert np.isfinite(hist.history['loss']).all()


def test_configs2_biwi_train_88_adam_b512():
    """BASELINE configs[2]: Model-88 training on the reference's own BIWI_train_features_88.npz
    (44 rows -> train_test_split(0.2, 42) = 35 train / 9 validation, train_88.py:290-297), the
    stoqa9pt create_model graph from its checkpoint, legacy Adam lr 2.8e-4, batch 512 (one partial
    batch per epoch), validation every epoch; weights, loss and val_loss after 20 epochs against the
    float64 oracle's fit on the same rows (dropout masks by the same counter hash)."""
    from hpe.data import train_test_split
    d = np.load(DATA + '/BIWI_train_features_88.npz')
    x = d['features'].reshape(-1, 1, 1, 88).astype(np.float32)
    y = d['poses'].reshape(-1, 1, 1, 3)
    tx, vx, ty, vy = train_test_split(x, y, test_size=0.2, random_state=42)
    assert (tx.shape[0], vx.shape[0]) == (35, 9)
    mc, w = fixture('stoqa9pt')
    hpe.set_seed(3)
    m = hpe.model_from_config(mc, w)
    m.compile(optimizer=keras.optimizers.Adam(learning_rate=2.8e-4), loss='mse', metrics=['mae'])
    epochs = 20
    hist = m.fit(tx, ty, batch_size=512, epochs=epochs, validation_data=(vx, vy), shuffle=False, verbose=0)
    g = K.Graph(mc, w)
    o = K.LegacyOptimizer('adam', 2.8e-4)
    vlosses = []
    for it in range(1, epochs + 1):
        K.train_step(g, o, tx, ty.reshape(-1, 3), drop_seed=hpe.random.dropout_seed(it))
        pv = g.forward(vx).detach().numpy().reshape(-1, 3)
        vlosses.append(float(np.mean((pv - vy.reshape(-1, 3)) ** 2)) + float(g.regularization().item()))
    got = m.weights_dict()
    for k in g.trainable:
        np.testing.assert_allclose(got[k], g.params[k].detach().numpy(), rtol=2e-4, atol=2e-5, err_msg=k)
    np.testing.assert_allclose(hist.history['val_loss'], vlosses, rtol=1e-4)
    assert np.isfinite(hist.history['loss']).all() and hist.history['loss'][-1] < hist.history['loss'][0]


def test_train_88_default_complex_on_biwi_enlarged():
    """train_88.py's own default graph: create_model_complex(1e-6, 1e-4)
    (Model-88/attention_model.py:97-169 -> the drop-in builder), legacy SGD lr 2.8e-4, batch 128
    (train_88.py:48,53,323,355-363), on the reference's training data BIWI_Train_Enlarged_features_88
    (the first 1,000 rows after train_test_split(0.2, 42), 8 steps per epoch, last batch partial),
    2 epochs in order, against the float64 oracle's fit on the same rows (dropout masks by the same
    counter hash): every weight within rtol 2e-4 / atol 2e-5."""
    import importlib.util
    import os
    from hpe.data import train_test_split
    d = np.load(DATA + '/BIWI_Train_Enlarged_features_88_0.7_1.npz')
    x = d['features'].reshape(-1, 1, 1, 88).astype(np.float32)
    y = d['poses'].reshape(-1, 1, 1, 3)
    tx, _, ty, _ = train_test_split(x, y, test_size=0.2, random_state=42)
    tx, ty = tx[:1000], ty[:1000]
    path = os.path.join(os.path.dirname(DATA), '..', '..', 'head-pose-estimation-model_amd', 'Model-88',
                        'attention_model.py')
    spec = importlib.util.spec_from_file_location('hpe_attention_model_88_t', path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    keras.backend.clear_session()
    hpe.set_seed(88)
    m = mod.create_model_complex(1e-6, 1e-4)
    m.compile(optimizer=keras.optimizers.SGD(learning_rate=2.8e-4), loss='mse', metrics=['mae'])
    w0 = m.weights_dict()
    hist = m.fit(tx, ty, batch_size=128, epochs=2, shuffle=False, verbose=0)
    g = K.Graph(m.model_config, w0)
    o = K.LegacyOptimizer('sgd', 2.8e-4)
    it = 0
    for _ in range(2):
        for b0 in range(0, tx.shape[0], 128):
            it += 1
            K.train_step(g, o, tx[b0:b0 + 128], ty[b0:b0 + 128].reshape(-1, 3), drop_seed=hpe.random.dropout_seed(it))
    got = m.weights_dict()
    for k in g.trainable:
        np.testing.assert_allclose(got[k], g.params[k].detach().numpy(), rtol=2e-4, atol=2e-5, err_msg=k)
    assert np.isfinite(hist.history['loss']).all()


@pytest.mark.parametrize('rid,opt,n', [('sqnu665j', 'adam', 128), ('stoqa9pt', 'sgd', 100),
                                       ('hrchr82r', 'adamax', 300), ('9w31h50k', 'adam', 77)])
def test_fused_reduce_optimizer_step_bit_identical(rid, opt, n):
    """hpe_reduce_optim_step (csrc/hpe_rowprog.hip reduce_optim_kernel: the slab reduction in
    reduce_kernel's order + the optimizer in one launch, fit's single-rank per-step path) against
    hpe_reduce + hpe_optim_step: gradient, parameters, moments and stats bit-identical over three
    steps (mlp2 programs and a generic row program)."""
    from hpe.engine import Engine
    from hpe import optimizers as O
    mc, w = fixture(rid)
    c = input_channels(mc)
    x = torch.from_numpy(features(n, c, seed=31).reshape(n, c)).cuda()
    y = torch.from_numpy(labels(n, seed=32).reshape(n, 3).astype(np.float32)).cuda()
    engs = [Engine(mc, w), Engine(mc, w)]
    o = O.get({'adam': 'Adam', 'sgd': 'SGD', 'adamax': 'Adamax'}[opt])
    o.learning_rate = 1e-3
    ng = engs[0].optim_grid()
    stats = [torch.zeros(2 + ng, dtype=torch.float32, device='cuda') for _ in engs]
    for it in range(3):
        for k, (e, st) in enumerate(zip(engs, stats)):
            g = e.gradient(x, y, 1, None, n, 1.0 / (n * 3), seed=it + 1, defer_reduce=(k == 1))
            if k == 1:
                assert g is None and e._pending is not None, 'small launch expected to defer its reduction'
            e.optimizer_step(o, st)
        a, b = engs
        np.testing.assert_array_equal(a.grad.cpu().numpy(), b.grad.cpu().numpy())
        np.testing.assert_array_equal(a.params.cpu().numpy(), b.params.cpu().numpy())
        np.testing.assert_array_equal(a.params_t.cpu().numpy(), b.params_t.cpu().numpy())
        np.testing.assert_array_equal(stats[0].cpu().numpy(), stats[1].cpu().numpy())
        if a.m is not None:
            np.testing.assert_array_equal(a.m.cpu().numpy(), b.m.cpu().numpy())
            np.testing.assert_array_equal(a.v.cpu().numpy(), b.v.cpu().numpy())


@pytest.mark.parametrize('rid,opt,bs,side', [('sqnu665j', 'adam', 128, 1), ('sqnu665j', 'sgd', 500, 1),
                                             ('9w31h50k', 'adamax', 77, 1), ('ker7z9mv', 'adam', 64, 1),
                                             ('hrchr82r', 'adam', 16, 4)])
def test_fit_steps_in_c_matches_python_loop(rid, opt, bs, side):
    """hpe_fit_steps (fit's per-step path with the step loop in C) against the Python step loop
    (HPE_FIT_STEPS=0): the same launches with the same arguments, so after 2 epochs every weight,
    moment and the loss history are bit-identical — mlp2 / residual-stack / generic row programs, a
    batch whose launch grid exceeds the fused reduce + optimizer launch (500), 4x4 maps."""
    import os
    mc, w = fixture(rid)
    c = input_channels(mc)
    n = 1000 if bs >= 128 else 300
    x = features(n, c, seed=41, h=side, w=side)
    y = labels(n, seed=42)
    prev = {k: os.environ.get(k) for k in ('HPE_FIT_STEPS', 'HPE_FIT_FUSED')}
    out = {}
    try:
        os.environ['HPE_FIT_FUSED'] = '0'
        for mode in ('0', '1'):
            os.environ['HPE_FIT_STEPS'] = mode
            hpe.set_seed(9)
            m = hpe.model_from_config(mc, w)
            m.compile(optimizer={'adam': keras.optimizers.Adam, 'sgd': keras.optimizers.SGD,
                                 'adamax': keras.optimizers.Adamax}[opt](learning_rate=1e-3),
                      loss='mse', metrics=['mae'])
            h = m.fit(x, y, batch_size=bs, epochs=2, shuffle=True, verbose=0)
            assert not m._last_fit_fused
            out[mode] = (m.weights_dict(), h.history['loss'], h.history['mae'])
    finally:
        for k, v in prev.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    for k, v in out['0'][0].items():
        np.testing.assert_array_equal(out['1'][0][k], v, err_msg=k)
    assert out['1'][1] == out['0'][1] and out['1'][2] == out['0'][2]
