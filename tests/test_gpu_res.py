"""GPU: the fused residual-stack kernels (csrc/hpe_res.hip) — train_88.py's default graph,
create_model_complex(reg, dr) (Model-88/attention_model.py:97-169), trained per step
(hpe_train_step -> res_train_kernel) and as one launch per epoch (hpe_fit_epoch -> res_fit_kernel).
Every GEMM runs on exact-fp32 MFMA, so the gradient is held to the float64 oracle at the fp32 level
(normwise 1e-5 of max |g|), and the fused epoch to the per-step path bit for bit."""
import importlib.util
import os

import numpy as np
import pytest
import torch

import hpe
from hpe import keras
from util import features, labels

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DATA = os.path.join(ROOT, 'tests', 'golden', 'data')


def _complex(reg=1e-6, dr=1e-4, opt=None, seed=88):
    """create_model_complex of the drop-in Model-88/attention_model.py, compiled as train_88.py:323-328."""
    path = os.path.join(ROOT, 'head-pose-estimation-model_amd', 'Model-88', 'attention_model.py')
    spec = importlib.util.spec_from_file_location('hpe_attention_model_88_res', path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    keras.backend.clear_session()
    hpe.set_seed(seed)
    m = mod.create_model_complex(reg, dr)
    m.compile(optimizer=opt or keras.optimizers.SGD(learning_rate=2.8e-4), loss='mse', metrics=['mae'])
    return m


def _grad64(mc, w, x, y, layout, seed):
    from test_gpu_parity import _data_grad64
    return _data_grad64(mc, w, x, y, layout, seed)


def test_complex_compiles_to_res_program():
    m = _complex()
    eng = m._eng()
    assert eng.program('train', 1).prog.kind == 'res'
    assert eng.program('train', 1).prog.info['blocks'] == 3


@pytest.mark.parametrize('n,side,dr,gather', [(128, 1, 1e-4, False), (203, 1, 0.3, False), (20, 3, 0.2, False),
                                              (77, 1, 0.1, True)])
def test_res_gradient_vs_float64_oracle(n, side, dr, gather):
    """One training launch (hpe_train_step + hpe_reduce) against the float64 oracle's autograd
    gradient with the same dropout masks: batch 128 (train_88.py's), a ragged 203 rows at a high
    dropout rate, 3x3 maps (P = 9: SpatialDropout per image and channel) and an index-gathered batch."""
    m = _complex(dr=dr)
    eng = m._eng()
    P = side * side
    assert eng.program('train', P).prog.kind == 'res'
    x = features(n, 88, seed=3, h=side, w=side)
    y = labels(n, seed=4)
    xt = torch.from_numpy(x.reshape(n * P, 88)).cuda()
    yt = torch.from_numpy(y.reshape(n, 3).astype(np.float32)).cuda()
    idx = None
    if gather:
        # rows of a permuted batch read through the image index, as fit gathers them
        perm = np.random.default_rng(5).permutation(n).astype(np.int32)
        idx = torch.from_numpy(perm).cuda()
        x, y = x[perm], y[perm]
    g = eng.gradient(xt, yt, P, idx, n, 1.0 / (n * P * 3), seed=11).cpu().numpy().astype(np.float64)
    g64 = _grad64(m.model_config, m.weights_dict(), x, y, eng.layout, 11)
    npt = eng.n_train
    scale = np.abs(g64).max()
    err = np.abs(g[:npt] - g64).max() / scale
    print('res n=%d P=%d dr=%g gather=%s: max |g - g64| / max |g64| = %.2e' % (n, P, dr, gather, err))
    assert err <= 1e-5, err
    # loss sums: sum e^2 and sum |e| of the step
    from oracle import keras_ref as K
    gr = K.Graph(m.model_config, m.weights_dict())
    p = gr.forward(x, training=True, drop_seed=11).detach().numpy().reshape(n, P, 3)
    e = p - y.reshape(n, 1, 3)
    np.testing.assert_allclose(g[npt], (e * e).sum(), rtol=1e-5)
    np.testing.assert_allclose(g[npt + 1], np.abs(e).sum(), rtol=1e-5)


def test_res_gradient_repeatable():
    """The partial gradients are summed in a fixed order (8-wave tree, fixed slab order): repeated
    launches on identical inputs are bit-identical (race screen)."""
    m = _complex()
    eng = m._eng()
    n = 1000
    x = torch.from_numpy(features(n, 88, seed=6).reshape(n, 88)).cuda()
    y = torch.from_numpy(labels(n, seed=7).reshape(n, 3).astype(np.float32)).cuda()
    ref = eng.gradient(x, y, 1, None, n, 1.0 / (n * 3), seed=2).cpu().numpy().copy()
    for _ in range(30):
        g = eng.gradient(x, y, 1, None, n, 1.0 / (n * 3), seed=2).cpu().numpy()
        assert np.array_equal(g, ref)


@pytest.mark.parametrize('opt,bs', [('sgd', 128), ('adam', 128), ('adamax', 96), ('adam', 300)])
def test_res_fused_epoch_matches_per_step_bit_for_bit(opt, bs):
    """fit's whole-epoch launch (res_fit_kernel: gradient, then the Keras legacy optimizer in LDS)
    against the per-step path (res_train_kernel on one workgroup + hpe_reduce_optim_step): the same
    gradient code, the same summation order and the same optimizer arithmetic, so after 3 epochs
    of BIWI_Train_Enlarged rows every weight is bit-identical."""
    d = np.load(DATA + '/BIWI_Train_Enlarged_features_88_0.7_1.npz')
    x = d['features'].reshape(-1, 1, 1, 88).astype(np.float32)[:700]
    y = d['poses'].reshape(-1, 1, 1, 3)[:700]
    mk = {'sgd': lambda: keras.optimizers.SGD(learning_rate=2.8e-4),
          'adam': lambda: keras.optimizers.Adam(learning_rate=2.8e-4),
          'adamax': lambda: keras.optimizers.Adamax(learning_rate=1e-3)}[opt]
    out = {}
    hist = {}
    prev = os.environ.get('HPE_FIT_FUSED')
    try:
        for mode in ('0', '1'):
            os.environ['HPE_FIT_FUSED'] = mode
            m = _complex(opt=mk(), seed=5)
            h = m.fit(x, y, batch_size=bs, epochs=3, shuffle=True, verbose=0)
            assert m._last_fit_fused == (mode == '1')
            out[mode] = m.weights_dict()
            hist[mode] = h.history['loss']
    finally:
        if prev is None:
            os.environ.pop('HPE_FIT_FUSED', None)
        else:
            os.environ['HPE_FIT_FUSED'] = prev
    for k, v in out['0'].items():
        np.testing.assert_array_equal(out['1'][k], v, err_msg=k)
    np.testing.assert_allclose(hist['1'], hist['0'], rtol=1e-5)
