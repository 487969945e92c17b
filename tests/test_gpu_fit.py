"""GPU: the whole-epoch launch (csrc/hpe_fit.hip, hpe_fit_epoch) that runs Keras fit's step loop
on the device for the reference's own regime — 1x1 maps, the create_model family, batch 128
(Model-96/train_96.py:134-140,175-183; Model-88/train_88.py:290-297,355-363).  Checked against the
float64 oracle's step-by-step fit (K.train_step, same batches, same dropout masks) and against the
per-step launch path (train_step + reduce + optimizer per step, HPE_FIT_FUSED=0)."""
import os

import numpy as np
import pytest
import torch

import hpe
from hpe import keras
from oracle import keras_ref as K
from util import features, fixture, labels

pytestmark = pytest.mark.gpu

OPT = {'adam': keras.optimizers.Adam, 'sgd': keras.optimizers.SGD, 'adamax': keras.optimizers.Adamax}


def _oracle_fit(mc, w, opt, lr, x, y, bs, epochs, perms):
    g = K.Graph(mc, w)
    o = K.LegacyOptimizer(opt, lr)
    it = 0
    for e in range(epochs):
        p = perms[e]
        for b0 in range(0, len(p), bs):
            it += 1
            b = p[b0:b0 + bs]
            K.train_step(g, o, x[b], y[b], drop_seed=hpe.random.dropout_seed(it))
    return g


def _model(src, F=360, act='tanh', dropout=0.0, l2=0.1, cin=96):
    keras.backend.clear_session()
    if src != 'new':
        mc, w = fixture(src)
        return hpe.model_from_config(mc, w)
    reg = keras.regularizers.l2(l2)
    inp = keras.Input(shape=(None, None, cin))
    h = keras.layers.Conv2D(F, 1, activation=act, kernel_regularizer=reg, bias_regularizer=reg)(inp)
    h = keras.layers.SpatialDropout2D(dropout)(h)
    o = keras.layers.Conv2D(3, 1, kernel_regularizer=reg, bias_regularizer=reg)(h)
    o = keras.layers.SpatialDropout2D(dropout)(o)
    return keras.Model(inp, o)


def _fit(m, opt, lr, x, y, bs, epochs, fused, shuffle=True):
    prev = os.environ.get('HPE_FIT_FUSED')
    os.environ['HPE_FIT_FUSED'] = '1' if fused else '0'
    try:
        hpe.set_seed(5)
        m.compile(optimizer=OPT[opt](learning_rate=lr), loss='mse', metrics=['mae'])
        h = m.fit(x, y, batch_size=bs, epochs=epochs, shuffle=shuffle, verbose=0)
    finally:
        if prev is None:
            os.environ.pop('HPE_FIT_FUSED')
        else:
            os.environ['HPE_FIT_FUSED'] = prev
    assert m._last_fit_fused == fused
    return h


CASES = [  # (model source, F, act, dropout, optimizer, lr, batch, rows, epochs)
    ('sqnu665j', 360, 'tanh', 0.0, 'adam', 2.8e-4, 128, 1000, 2),       # create_model(360), l2 0.1
    ('stoqa9pt', 64, 'softsign', 1e-4, 'adam', 2.8e-4, 256, 700, 2),    # Model-88 88-64-3, dropout
    ('new', 384, 'tanh', 0.2, 'adam', 2.8e-4, 128, 450, 2),             # create_model(384): 12 workgroups
    ('new', 256, 'relu', 0.1, 'adamax', 2.8e-4, 200, 601, 2),           # runtime activation, ragged batch
    ('new', 16, 'tanh', 0.0, 'sgd', 0.05, 128, 300, 3),                 # one workgroup, SGD
    ('new', 100, 'elu', 0.3, 'adam', 1e-3, 32, 97, 2),                  # tiny batches, partial last
    # batches beyond 256: X re-gathered for the backward, partial table over the X slots
    ('sqnu665j', 360, 'tanh', 0.0, 'adam', 2.8e-4, 512, 1100, 2),       # p1 b512; last batch 76
    ('stoqa9pt', 64, 'softsign', 1e-4, 'adam', 2.8e-4, 512, 1300, 2),   # configs[2]: Model-88, Adam, b512
    ('new', 384, 'tanh', 0.1, 'sgd', 0.01, 300, 901, 2),                # 12 workgroups, batch 300
]


@pytest.mark.parametrize('src,F,act,dropout,opt,lr,bs,n,epochs', CASES)
def test_fused_epoch_matches_oracle_and_per_step(src, F, act, dropout, opt, lr, bs, n, epochs):
    m0 = _model(src, F, act, dropout)
    cin = m0.model_config['config']['layers'][0]['config']['batch_input_shape'][-1]
    w0 = m0.weights_dict()
    x = features(n, cin, seed=n)
    y = labels(n, seed=n + 1)
    mf = hpe.model_from_config(m0.model_config, w0)
    hf = _fit(mf, opt, lr, x, y, bs, epochs, fused=True)
    mp = hpe.model_from_config(m0.model_config, w0)
    hp = _fit(mp, opt, lr, x, y, bs, epochs, fused=False)
    rng = np.random.RandomState(5)
    perms = [rng.permutation(n) for _ in range(epochs)]
    g = _oracle_fit(m0.model_config, w0, opt, lr, x, y, bs, epochs, perms)
    wf, wp = mf.weights_dict(), mp.weights_dict()
    for k in g.trainable:
        ref = g.params[k].detach().numpy()
        np.testing.assert_allclose(wf[k], ref, rtol=2e-4, atol=2e-5, err_msg='fused ' + k)
        np.testing.assert_allclose(wf[k], wp[k], rtol=2e-4, atol=2e-5, err_msg='fused vs per-step ' + k)
    np.testing.assert_allclose(hf.history['loss'], hp.history['loss'], rtol=1e-4)
    np.testing.assert_allclose(hf.history['mae'], hp.history['mae'], rtol=1e-4)
    assert mf._eng().iterations == mp._eng().iterations == epochs * -(-n // bs)
    # the optimizer state written back at the epoch end is the per-step path's
    if opt != 'sgd':
        mm = mp._eng().m.cpu().numpy()
        np.testing.assert_allclose(mf._eng().m.cpu().numpy(), mm, rtol=2e-3, atol=1e-6 * np.abs(mm).max())


def test_fused_epoch_fp16_overflow_reruns_exact():
    """A feature beyond the split's data range (|x| >= 64) flags the epoch; it is re-run on the
    exact-fp32 path from the saved state and matches the per-step path (which falls back per step)."""
    m0 = _model('sqnu665j')
    w0 = m0.weights_dict()
    x = features(300, 96, seed=9)
    x[17, 0, 0, 5] = 100.0
    y = labels(300, seed=10)
    mf = hpe.model_from_config(m0.model_config, w0)
    _fit(mf, 'adam', 2.8e-4, x, y, 128, 2, fused=True)
    mp = hpe.model_from_config(m0.model_config, w0)
    _fit(mp, 'adam', 2.8e-4, x, y, 128, 2, fused=False)
    wf, wp = mf.weights_dict(), mp.weights_dict()
    for k in wf:
        assert np.isfinite(wf[k]).all()
        np.testing.assert_allclose(wf[k], wp[k], rtol=2e-4, atol=2e-5, err_msg=k)


def test_fused_epoch_reference_data_train_96():
    """train_96.py's own loop shape on the reference's substitute data (BIWI_Train_Enlarged_96,
    1,643 rows -> 1,314 / 329 split): create_model(360) from the sqnu665j checkpoint, batch 128,
    validation every epoch — fused and per-step give the same history."""
    from util import DATA
    d = np.load(DATA + '/BIWI_Train_Enlarged_features_96_0.7_1.npz')
    xa, ya = d['features'].reshape(-1, 1, 1, 96).astype(np.float32), d['poses'].reshape(-1, 1, 1, 3)
    from hpe.data import train_test_split
    tx, vx, ty, vy = train_test_split(xa, ya, test_size=0.2, random_state=42)
    m0 = _model('sqnu665j')
    w0 = m0.weights_dict()
    hs = []
    for fused in (True, False):
        os.environ['HPE_FIT_FUSED'] = '1' if fused else '0'
        try:
            hpe.set_seed(42)
            m = hpe.model_from_config(m0.model_config, w0)
            m.compile(optimizer=keras.optimizers.Adam(learning_rate=2.8e-4), loss='mse', metrics=['mae'])
            hs.append(m.fit(tx, ty, batch_size=128, epochs=3, validation_data=(vx, vy), verbose=0))
            assert m._last_fit_fused == fused
        finally:
            os.environ.pop('HPE_FIT_FUSED')
    for k in ('loss', 'mae', 'val_loss', 'val_mae'):
        np.testing.assert_allclose(hs[0].history[k], hs[1].history[k], rtol=1e-4, err_msg=k)


def test_fused_epoch_timeout_rolls_back_to_per_step():
    """a workgroup-exchange timeout (forced: HPE_FIT_FORCE_TIMEOUT=1) leaves the
    workgroups at different steps; the engine restores the saved parameters / Adam state, disables
    the fused path and runs the epoch per step -- the result is the per-step path's."""
    m0 = _model('sqnu665j')
    w0 = m0.weights_dict()
    x = features(400, 96, seed=21)
    y = labels(400, seed=22)
    mf = hpe.model_from_config(m0.model_config, w0)
    os.environ['HPE_FIT_FORCE_TIMEOUT'] = '1'
    try:
        hpe.set_seed(5)
        mf.compile(optimizer=OPT['adam'](learning_rate=2.8e-4), loss='mse', metrics=['mae'])
        with pytest.warns(UserWarning, match='timed out'):
            hf = mf.fit(x, y, batch_size=128, epochs=2, verbose=0)
    finally:
        os.environ.pop('HPE_FIT_FORCE_TIMEOUT')
    assert mf._last_fit_fused is False and mf._eng()._fit_disabled
    mp = hpe.model_from_config(m0.model_config, w0)
    hp = _fit(mp, 'adam', 2.8e-4, x, y, 128, 2, fused=False)
    wf, wp = mf.weights_dict(), mp.weights_dict()
    for k in wf:
        np.testing.assert_array_equal(wf[k], wp[k], err_msg=k)
    np.testing.assert_allclose(hf.history['loss'], hp.history['loss'], rtol=1e-6)
    assert mf._eng().iterations == mp._eng().iterations == 2 * 4
