"""In-process Keras .h5 reader (hpe/h5io.py).

Golden: four of the reference's checkpoints, committed as data under tests/golden/h5/, against the
h5py conversions of the same files (tests/golden/models/*.json / .npz, tests/golden/make_fixtures.py).
Three are the files Keras wrote (Model-96 hrchr82r, Model-96 0g73t16n with its Adam state, Model-88
stoqa9pt with its SGD state); the fourth, Model-88 ker7z9mv (SE + MHA with Lambda layers), was
rewritten by this repo's own writer to drop the Lambda bytecode (tests/golden/strip_h5_bytecode.py).
The Keras-written ker7z9mv is kept too, under tests/golden/h5_keras/, with only the Lambda bytecode
overwritten in place by a same-length placeholder (tests/golden/patch_h5_lambda.py): every other
byte is the file libhdf5 wrote.  When /root/reference is present (the build container) every one of
its 688 .h5 files is parsed and each fixture exemplar compared.
"""
import glob
import json
import os

import numpy as np
import pytest

from hpe import h5io
from util import fixture

H5 = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'h5')
H5_KERAS = os.path.join(os.path.dirname(H5), 'h5_keras')
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


def test_reader_on_keras_written_se_mha_lambda_file():
    """The Keras-written SE + MHA + Lambda checkpoint (bytecode overwritten in place): the same
    graph, weights and optimizer state as the h5py conversion and as the rewritten fixture."""
    p = os.path.join(H5_KERAS, 'ker7z9mv.h5')
    mc, w, opt = h5io.read_keras_h5(p, with_optimizer=True)
    ref_mc, ref_w = fixture('ker7z9mv')
    assert mc == ref_mc
    assert sorted(w) == sorted(ref_w)
    for k in ref_w:
        np.testing.assert_array_equal(w[k], ref_w[k], err_msg=k)
    _, _, opt2 = h5io.read_keras_h5(os.path.join(H5, 'ker7z9mv.h5'), with_optimizer=True)
    assert list(opt) == list(opt2)
    for k in opt:
        np.testing.assert_array_equal(np.asarray(opt[k]), np.asarray(opt2[k]), err_msg=k)
    assert h5io.read_training_config(p) == h5io.read_training_config(os.path.join(H5, 'ker7z9mv.h5'))


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


# ---- writer (Model.save('x.h5'), ModelCheckpoint) ---------------------------------------------
def _layers_of(mc, w):
    out = []
    for l in mc['config']['layers']:
        ln = l['name']
        ws = [(k[len(ln) + 1:] + ':0' if l['class_name'] == 'Functional' else k + ':0', a)
              for k, a in w.items() if k.startswith(ln + '/')]
        out.append((ln, ws))
    return out


def _tree(f, addr=None, path=''):
    """{path: sorted attr names} of every object in a file (our reader), for structure checks."""
    addr = f.root if addr is None else addr
    out = {path or '/': sorted(f.attrs(addr))}
    ch = f.children(addr)
    for n, a in (ch or {}).items():
        out.update(_tree(f, a, path + '/' + n))
    return out


@pytest.mark.parametrize('rid', IDS)
def test_writer_roundtrip_fixture(rid, tmp_path):
    src = os.path.join(H5, rid + '.h5')
    mc, w, opt = h5io.read_keras_h5(src, with_optimizer=True)
    out = str(tmp_path / 'x.h5')
    h5io.write_keras_h5(out, mc, _layers_of(mc, w), h5io.read_training_config(src),
                        [(k + ':0', v) for k, v in opt.items()] or None)
    mc2, w2, opt2 = h5io.read_keras_h5(out, with_optimizer=True)
    assert mc2 == mc and list(w2) == list(w)
    for k in w:
        np.testing.assert_array_equal(w2[k], w[k])
        assert w2[k].dtype == w[k].dtype
    assert list(opt2) == list(opt)
    for k in opt:
        assert np.asarray(opt2[k]).shape == np.asarray(opt[k]).shape
        np.testing.assert_array_equal(opt2[k], opt[k])
    assert h5io.read_training_config(out) == h5io.read_training_config(src)
    # same objects and attribute names as the file Keras wrote (our writer adds the
    # top_level_model_weights group Keras 2.13.1 writes; older files may lack it)
    t_src, t_out = _tree(h5io._File(src)), _tree(h5io._File(out))
    t_out.pop('/model_weights/top_level_model_weights', None)
    t_src.pop('/model_weights/top_level_model_weights', None)
    assert t_out == t_src


def _h5py_python():
    p = '/opt/conda/bin/python3.9'
    if not os.path.exists(p):
        return None
    import subprocess
    r = subprocess.run([p, '-c', 'import h5py'], capture_output=True)
    return p if r.returncode == 0 else None


@pytest.mark.skipif(_h5py_python() is None, reason='no h5py interpreter (build container only)')
def test_writer_output_reads_in_h5py(tmp_path):
    """Independent check with libhdf5 itself (h5py 3.3 of /opt/conda, present in the build
    container only): every attribute and dataset of a written checkpoint reads back."""
    import subprocess
    src = os.path.join(H5, '0g73t16n.h5')
    mc, w, opt = h5io.read_keras_h5(src, with_optimizer=True)
    out = str(tmp_path / 'x.h5')
    h5io.write_keras_h5(out, mc, _layers_of(mc, w), h5io.read_training_config(src),
                        [(k + ':0', v) for k, v in opt.items()])
    script = r'''
import h5py, json, sys, numpy as np
f = h5py.File(sys.argv[1], 'r')
res = {'attrs': {k: str(v) for k, v in f.attrs.items()}, 'data': {}, 'gattrs': {}}
def visit(n, o):
    if isinstance(o, h5py.Dataset):
        a = np.asarray(o); res['data'][n] = [list(a.shape), str(a.dtype), float(np.asarray(a, np.float64).sum())]
    else:
        res['gattrs'][n] = {k: [str(x) for x in np.atleast_1d(v)] for k, v in o.attrs.items()}
f.visititems(visit)
print(json.dumps(res))
'''
    r = subprocess.run([_h5py_python(), '-c', script, out], capture_output=True, text=True, check=True)
    res = json.loads(r.stdout)
    assert json.loads(res['attrs']['model_config']) == mc
    assert res['attrs']['keras_version'] == '2.13.1' and res['attrs']['backend'] == 'tensorflow'
    assert res['gattrs']['model_weights']['layer_names'] == [l['name'] for l in mc['config']['layers']]
    for k, a in w.items():
        ln = k.split('/')[0]
        shape, dt, s = res['data']['model_weights/%s/%s:0' % (ln, k)]
        assert tuple(shape) == a.shape and dt == 'float32'
        assert s == pytest.approx(float(a.astype(np.float64).sum()), rel=1e-12, abs=1e-12)
    shape, dt, s = res['data']['optimizer_weights/Adam/iter:0']
    assert shape == [] and dt == 'int64' and s == float(opt['Adam/iter'])


def test_model_save_h5_and_load_model_compile(tmp_path):
    """Model.save('<id>.h5') (ModelCheckpoint's format) -> load_model: same graph, weights,
    optimizer class / hyper-parameters (float32-rounded like Keras's training_config)."""
    import hpe
    from hpe import keras
    hpe.set_seed(3)
    keras.backend.clear_session()
    inp = keras.Input(shape=(None, None, 96))
    h = keras.layers.Conv2D(16, 1, activation='tanh')(inp)
    out = keras.layers.Conv2D(3, 1)(keras.layers.SpatialDropout2D(0.1)(h))
    m = keras.Model(inp, out)
    m.compile(optimizer=keras.optimizers.Adamax(learning_rate=2.8e-4), loss='mse', metrics=['mae'])
    p = str(tmp_path / 'run' / 'abc12345.h5')
    m.save(p)
    assert open(p, 'rb').read(8) == b'\x89HDF\r\n\x1a\n'
    m2 = hpe.load_model(p)
    assert m2.model_config == m.model_config
    for a, b in zip(m.get_weights(), m2.get_weights()):
        np.testing.assert_array_equal(a, b)
    assert type(m2.optimizer).__name__ == 'Adamax'
    assert m2.optimizer.learning_rate == float(np.float32(2.8e-4))
    tc = h5io.read_training_config(p)
    assert tc['optimizer_config']['config']['learning_rate'] == float(np.float32(2.8e-4))
    _, _, opt = h5io.read_keras_h5(p, with_optimizer=True)
    assert list(opt) == ['Adamax/iter']  # no steps taken yet: iterations only
    m3 = hpe.load_model(p, compile=False)
    assert m3.optimizer is None


def test_load_model_restores_reference_adam_state():
    import hpe
    m = hpe.load_model(os.path.join(H5, '0g73t16n.h5'))
    assert type(m.optimizer).__name__ == 'Adam'
    _, _, opt = h5io.read_keras_h5(os.path.join(H5, '0g73t16n.h5'), with_optimizer=True)
    assert m._pending_opt['iter'] == int(opt['Adam/iter'])
    # re-saving without touching the device writes the same optimizer state back
    state = dict(m._optimizer_state())
    for k, v in opt.items():
        np.testing.assert_array_equal(state[k + ':0'], v)


@pytest.mark.gpu
def test_gpu_checkpoint_resume_is_exact(tmp_path):
    """fit 2 epochs, save .h5 (weights + Adam m/v/iter), load, fit 2 more == fit 4 straight."""
    import hpe
    from hpe import keras
    rng = np.random.default_rng(5)
    x = np.maximum(0.0, 0.6 * rng.standard_normal((300, 1, 1, 96)) - 0.3).astype(np.float32)
    y = (20 * rng.standard_normal((300, 1, 1, 3))).astype(np.float32)

    def build():
        hpe.set_seed(11)
        keras.backend.clear_session()
        inp = keras.Input(shape=(None, None, 96))
        h = keras.layers.Conv2D(32, 1, activation='tanh', kernel_regularizer=keras.regularizers.l2(1e-3))(inp)
        m = keras.Model(inp, keras.layers.Conv2D(3, 1)(h))
        m.compile(optimizer=keras.optimizers.Adam(learning_rate=1e-3), loss='mse', metrics=['mae'])
        return m
    a = build()
    a.fit(x, y, batch_size=64, epochs=4, shuffle=False, verbose=0)
    b = build()
    b.fit(x, y, batch_size=64, epochs=2, shuffle=False, verbose=0)
    p = str(tmp_path / 'ck.h5')
    b.save(p)
    c = hpe.load_model(p)
    c.fit(x, y, batch_size=64, epochs=2, shuffle=False, verbose=0)
    for wa, wc in zip(a.get_weights(), c.get_weights()):
        np.testing.assert_array_equal(wa, wc)


def test_no_reference_bytecode_in_committed_fixtures():
    """reference Lambda bytecode must not travel in any form.  Every committed .h5 /
    .json fixture's Lambda 'function' field is the stripped placeholder (raw attribute, before the
    reader's own stripping), and no file holds a base64 marshalled code object (0xe3 header)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        'strip_h5_bytecode', os.path.join(os.path.dirname(H5), 'strip_h5_bytecode.py'))
    sb = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(sb)
    n_lambda = 0
    for p in glob.glob(os.path.join(H5, '*.h5')) + glob.glob(os.path.join(H5_KERAS, '*.h5')):
        fns = sb.lambda_functions(sb.raw_model_config(p))
        n_lambda += len(fns)
        # our writer's plain placeholder, or Keras's [code, defaults, closure] with code patched
        assert all(f == '<bytecode stripped>' or (isinstance(f, list) and f[0] == '<bytecode stripped>')
                   for f in fns), p
    for p in glob.glob(os.path.join(MODELS, '*.json')):
        with open(p) as fh:
            d = json.load(fh)
        mc = d.get('model_config', d)
        if isinstance(mc, dict):
            assert all(f == '<bytecode stripped>' for f in sb.lambda_functions(mc)), p
    assert n_lambda >= 4                     # ker7z9mv's reshape_flat / reshape_back, both files
    for p in (glob.glob(os.path.join(H5, '*.h5')) + glob.glob(os.path.join(H5_KERAS, '*.h5'))
              + glob.glob(os.path.join(MODELS, '*.json'))):
        with open(p, 'rb') as fh:
            raw = fh.read()
        assert b'4wEAAAAA' not in raw and b'4wAAAAAA' not in raw, p
