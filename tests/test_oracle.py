"""CPU: the oracle against the reference's own data (BASELINE.md goldens computed from the
reference's TF-trained checkpoints), sklearn's real train_test_split, and internal consistency."""
import numpy as np
import pytest
import torch

from oracle import keras_ref as K
from util import DATA, MODELS, fixture, index

GOLDEN = [
    ('stoqa9pt', 'AFLW2000_features_88_0.7_1.npz', (39.655, 50.258, 44.566), 44.8263),
    ('stoqa9pt', 'AFLW2000_Enlarged_features_88_0.7_1.npz', (6.535, 9.810, 7.085), 7.8100),
    ('stoqa9pt', 'BIWI_Test_Enlarged_features_88_0.7_1.npz', (3.181, 3.881, 3.275), 3.4456),
    ('ker7z9mv', 'AFLW2000_Enlarged_features_88_0.7_1.npz', (6.795, 9.957, 7.225), 7.9921),
    ('9w31h50k', 'AFLW2000_Enlarged_features_88_0.7_1.npz', None, 8.3447),
    ('hrchr82r', 'AFLW2000_features_96_0.7_1.npz', (7.216, 9.920, 6.956), 8.0307),
    ('model_runid_hrchr82r', 'AFLW2000_features_96_0.7_1.npz', (7.216, 9.920, 6.956), 8.0307),
    ('sqnu665j', 'AFLW2000_features_96_0.7_1.npz', (7.555, 9.011, 6.782), 7.7826),
    ('o6e5xpan', 'AFLW2000_features_96_0.7_1.npz', (7.064, 9.439, 6.663), 7.7222),
]


@pytest.mark.parametrize('rid,ds,per_angle,avg', GOLDEN)
def test_oracle_reproduces_golden_mae(rid, ds, per_angle, avg):
    g, _ = K.load_fixture(MODELS + '/' + rid)
    d = np.load(DATA + '/' + ds)
    x, y = d['features'], d['poses']
    p = g.forward(x.reshape(-1, 1, 1, x.shape[1])).detach().numpy().reshape(-1, 3)
    m = K.evaluate_head_pose(p, y)
    assert abs(m['MAE']['average'] - avg) < 1e-4
    if per_angle:
        got = (m['MAE']['yaw'], m['MAE']['pitch'], m['MAE']['roll'])
        assert np.allclose(got, per_angle, atol=6e-4)


def test_oracle_fp32_vs_fp64_drift():
    g64, _ = K.load_fixture(MODELS + '/hrchr82r')
    g32, _ = K.load_fixture(MODELS + '/hrchr82r', dtype=torch.float32)
    d = np.load(DATA + '/AFLW2000_features_96_0.7_1.npz')
    x = d['features'].reshape(-1, 1, 1, 96)
    a = g64.forward(x).detach().numpy()
    b = g32.forward(x).detach().numpy()
    assert np.abs(a - b).max() < 1e-4


@pytest.mark.parametrize('n', [44, 1643, 10284, 12000])
def test_split_matches_sklearn(n):
    sk = pytest.importorskip('sklearn.model_selection')
    idx = np.arange(n)
    tr, te = sk.train_test_split(idx, test_size=0.2, random_state=42)
    otr, ote = K.split_indices(n, 0.2, 42)
    assert np.array_equal(tr, otr) and np.array_equal(te, ote)


def test_flatten_and_noflatten_checkpoints_agree():
    """model_runid_hrchr82r (1x1 input + Flatten) and hrchr82r (NoFlatten): identical predictions,
    the claim InputShapeConvertor.validate_conversion makes (Model-96/InputShapeConvertor.py:205)."""
    a, _ = K.load_fixture(MODELS + '/hrchr82r')
    b, _ = K.load_fixture(MODELS + '/model_runid_hrchr82r')
    x = np.random.default_rng(0).random((50, 1, 1, 96)).astype(np.float32)
    np.testing.assert_allclose(a.forward(x).detach().numpy().reshape(-1, 3),
                               b.forward(x).detach().numpy().reshape(-1, 3), rtol=1e-5, atol=1e-5)


def test_unified_model_embeds_selected_heads():
    """The fused BlazeFace graph's heads are bit-identical to stoqa9pt / hrchr82r."""
    u = dict(np.load(MODELS + '/reg1-stoqa9pt-reg2-hrchr82r-selected.npz'))
    s = dict(np.load(MODELS + '/stoqa9pt.npz'))
    h = dict(np.load(MODELS + '/hrchr82r.npz'))
    for k, v in s.items():
        assert np.array_equal(u['model/' + k], v)
    for k, v in h.items():
        assert np.array_equal(u['model_10/' + k], v)


def test_dropout_hash_restatements_agree():
    """The emulator's copy of the kernels' dropout hash (tests/rowprog_emu.py) equals the oracle's,
    over seeds, ordinals, images past 2^32 and channels."""
    import rowprog_emu as E
    rng = np.random.default_rng(0)
    img = rng.integers(0, 1 << 40, 5000, dtype=np.uint64)
    ch = rng.integers(0, 1024, 5000, dtype=np.uint64)
    for seed, did in ((0, 0), (123456789, 3), ((1 << 64) - 5, 17)):
        np.testing.assert_array_equal(E._hash(seed, did, img, ch), K.dropout_hash(seed, did, img, ch))


def test_dropout_hash_rate():
    m = K.dropout_mask(123, 0, 4096, 64, 0.3)
    keep = (m > 0).mean()
    assert abs(keep - 0.7) < 0.01
    assert np.allclose(m[m > 0], 1 / np.float32(0.7))


def test_every_fixture_runs_forward():
    for rid in index():
        if rid.startswith('reg1'):
            continue
        g, meta = K.load_fixture(MODELS + '/' + rid)
        c = meta['model_config']['config']['layers'][0]['config']['batch_input_shape'][-1]
        out = g.forward(np.ones((2, 1, 1, c), np.float32))
        assert np.isfinite(out.detach().numpy()).all(), rid


def test_legacy_adam_matches_closed_form():
    """Legacy Keras Adam (TF ApplyAdam functor) on a scalar for 3 steps."""
    w = {'w': torch.tensor([1.0], dtype=torch.float64)}
    opt = K.LegacyOptimizer('adam', 0.1)
    m = v = 0.0
    x = 1.0
    for t in range(1, 4):
        g = 2 * x
        opt.apply(w, {'w': torch.tensor([g], dtype=torch.float64)})
        m += (g - m) * 0.1
        v += (g * g - v) * 0.001
        x -= 0.1 * np.sqrt(1 - 0.999 ** t) / (1 - 0.9 ** t) * m / (np.sqrt(v) + 1e-7)
        assert abs(w['w'].item() - x) < 1e-12
