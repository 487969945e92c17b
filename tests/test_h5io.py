"""In-process Keras .h5 reader (hpe/h5io.py).

Golden: four of the reference's own checkpoints, committed as data under tests/golden/h5/
(Model-96 hrchr82r, Model-96 0g73t16n with its Adam state, Model-88 stoqa9pt with its SGD state,
Model-88 ker7z9mv SE + MHA with Lambda layers), against the h5py conversions of the same files
(tests/golden/models/*.json / .npz, tests/golden/make_fixtures.py).  When /root/reference is present
(the build container) every one of its 688 .h5 files is parsed and each fixture exemplar compared.
"""
import glob
import json
import os

import numpy as np
import pytest

from hpe import h5io
from util import fixture

H5 = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'h5')
MODELS = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'models')
IDS = sorted(os.path.basename(p)[:-3] for p in glob.glob(os.path.join(H5, '*.h5')))


def test_h5_fixtures_present():
    assert {'hrchr82r', 'stoqa9pt', 'ker7z9mv', '0g73t16n'} <= set(IDS)


@pytest.mark.parametrize('rid', IDS)
def test_reader_matches_h5py_conversion(rid):
    mc, w = h5io.read_keras_h5(os.path.join(H5, rid + '.h5'))
    ref_mc, ref_w = fixture(rid)
    assert mc == ref_mc
    assert sorted(w) == sorted(ref_w)
    for k in ref_w:
        assert w[k].dtype == np.float32
        np.testing.assert_array_equal(w[k], ref_w[k], err_msg=k)


@pytest.mark.parametrize('rid', ['0g73t16n', 'stoqa9pt'])
def test_reader_optimizer_state(rid):
    _, _, opt = h5io.read_keras_h5(os.path.join(H5, rid + '.h5'), with_optimizer=True)
    ref = np.load(os.path.join(MODELS, rid + '.opt.npz'))
    assert sorted(opt) == sorted(ref.files)
    for k in ref.files:
        np.testing.assert_array_equal(np.asarray(opt[k]), ref[k], err_msg=k)


def test_load_model_h5_builds_the_graph():
    import hpe
    m = hpe.load_model(os.path.join(H5, 'hrchr82r.h5'))
    assert m.count_params() == 3683
    mc, _ = fixture('hrchr82r')
    assert m.model_config['config']['layers'] == mc['config']['layers']


def test_not_hdf5_and_missing_file():
    with pytest.raises(FileNotFoundError):
        import hpe
        hpe.load_model('/nonexistent/model.h5')
    with pytest.raises(h5io.H5Error):
        h5io.read_keras_h5(os.path.join(MODELS, 'index.json'))


@pytest.mark.skipif(not os.path.isdir('/root/reference'), reason='reference checkpoints absent')
def test_every_reference_checkpoint_parses_and_exemplars_match():
    files = {os.path.basename(p)[:-3]: p for p in glob.glob('/root/reference/**/*.h5', recursive=True)}
    assert len(files) >= 600
    for rid, p in files.items():
        h5io.read_keras_h5(p)
    idx = json.load(open(os.path.join(MODELS, 'index.json')))['models']
    for rid in idx:
        mc, w = h5io.read_keras_h5(files[rid])
        ref_mc, ref_w = fixture(rid)
        assert mc == ref_mc, rid
        assert sorted(w) == sorted(ref_w), rid
        for k in ref_w:
            np.testing.assert_array_equal(w[k], ref_w[k], err_msg='%s %s' % (rid, k))


@pytest.mark.gpu
@pytest.mark.parametrize('rid', ['hrchr82r', 'stoqa9pt', 'ker7z9mv'])
def test_gpu_predict_from_h5_matches_oracle(rid):
    import hpe
    from oracle import keras_ref as K
    m = hpe.load_model(os.path.join(H5, rid + '.h5'))
    mc, w = fixture(rid)
    c = mc['config']['layers'][0]['config']['batch_input_shape'][-1]
    x = np.maximum(0.0, 0.6 * np.random.default_rng(1).standard_normal((40, 1, 1, c)) - 0.3).astype(np.float32)
    ref = K.Graph(mc, w).forward(x).detach().numpy()
    np.testing.assert_allclose(m.predict(x), ref, rtol=1e-5, atol=1e-4)
