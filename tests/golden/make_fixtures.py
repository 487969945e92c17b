"""Convert the reference's Keras ``.h5`` checkpoints and ``.npz`` datasets into committed fixtures.

Runs ONLY in the survey container, under ``/opt/conda/bin/python3.9`` (the one interpreter here
that has ``h5py``); the GPU box never runs it.  HDF5 is read purely as data: array datasets and
the ``model_config`` JSON attribute.  ``Lambda`` layers carry marshalled Python bytecode in their
config; it is dropped here and never executed (the executors recognise the two reshape lambdas of
``Model-88/attention_model.py:43-50,66-72`` by their position in the graph).

Outputs (all small):
  tests/golden/models/<run_id>.json   Keras ``model_config`` (bytecode stripped)
  tests/golden/models/<run_id>.npz    weights, keys ``<layer>/<weight>`` (``:0`` suffix removed)
  tests/golden/models/<run_id>.opt.npz  legacy-optimizer state (only for OPT_STATE ids)
  tests/golden/models/index.json      run_id -> {dir, signature, n_params}
  tests/golden/data/*.npz             the reference datasets used by the parity tests (copied)

One exemplar per distinct graph signature (smallest file) plus every checkpoint named in
BASELINE.md, so the forward parity tests cover every layer type the 684 checkpoints use.  Round 1
skipped the 16 signatures whose smallest checkpoint exceeds 400 kB; round 2 converts them too
(``--only-missing`` converts only checkpoints without a fixture, leaving the committed ones
byte-identical).
"""
import glob
import json
import os
import shutil
import sys

import h5py
import numpy as np

REF = '/root/reference'
HERE = os.path.dirname(os.path.abspath(__file__))
OUT_M = os.path.join(HERE, 'models')
OUT_D = os.path.join(HERE, 'data')

NAMED = ['stoqa9pt', 'ker7z9mv', '9w31h50k', '4121t6zb', 'hrchr82r', 'model_runid_hrchr82r',
         'sqnu665j', 'o6e5xpan', '0g73t16n', 'cl4obelj']
OPT_STATE = ['0g73t16n', 'stoqa9pt']
MAX_BYTES = 2_000_000
# the four fused BlazeFace + regressor graphs (BlazePoser/UnifiedModels, blazeFaceDetectorH5.py:97-101)
UNIFIED = ['reg1-stoqa9pt-reg2-hrchr82r-selected', 'reg1-stoqa9pt-reg2-cl4obelj', 'reg1-9w31h50k-reg2-cl4obelj',
           'reg1-4121t6zb-reg2-cl4obelj']
DATASETS = ['AFLW2000_features_88_0.7_1.npz', 'AFLW2000_features_96_0.7_1.npz',
            'AFLW2000_Enlarged_features_88_0.7_1.npz', 'BIWI_train_features_88.npz',
            'BIWI_test_features_88.npz', 'BIWI_Test_Enlarged_features_88_0.7_1.npz',
            'BIWI_Train_Enlarged_features_96_0.7_1.npz', 'BIWI_Test_Enlarged_features_96_0.7_1.npz',
            'BIWI_Train_Enlarged_features_88_0.7_1.npz']   # Model-88's training set (train_88.py:270)


def strip(mc):
    for l in mc['config']['layers']:
        if l['class_name'] == 'Lambda':
            l['config']['function'] = '<bytecode stripped>'
    return mc


def signature(mc):
    parts = []
    for l in mc['config']['layers']:
        c = l['config']
        parts.append('%s:%s:%s:%s:%s' % (l['class_name'], c.get('filters', c.get('units')),
                                         c.get('kernel_size'), c.get('activation'),
                                         json.dumps(l.get('inbound_nodes'))))
    return '|'.join(parts)


def weights(g, pre=''):
    out = {}
    for k, v in g.items():
        if isinstance(v, h5py.Dataset):
            out[(pre + k).replace(':0', '')] = np.asarray(v)
        else:
            out.update(weights(v, pre + k + '/'))
    return out


def convert(path, run_id):
    f = h5py.File(path, 'r')
    mc = strip(json.loads(f.attrs['model_config']))
    w = {}
    for lname in f['model_weights'].attrs['layer_names']:
        lname = lname.decode() if isinstance(lname, bytes) else lname
        g = f['model_weights'][lname]
        for wn in g.attrs['weight_names']:
            wn = wn.decode() if isinstance(wn, bytes) else wn
            # keys are '<layer>/<sublayer...>/<var>' as Keras stores them, ':0' dropped; a
            # nested Functional layer's weights get its own name in front ('model/conv2d/kernel')
            key = wn.replace(':0', '')
            if not key.startswith(lname + '/'):
                key = lname + '/' + key
            w[key] = np.asarray(g[wn]).astype(np.float32)
    with open(os.path.join(OUT_M, run_id + '.json'), 'w') as fh:
        json.dump({'model_config': mc,
                   'keras_version': str(f.attrs.get('keras_version', b'')),
                   'source': os.path.relpath(path, REF)}, fh, indent=0)
    np.savez_compressed(os.path.join(OUT_M, run_id + '.npz'), **w)
    if run_id in OPT_STATE and 'optimizer_weights' in f:
        ow = weights(f['optimizer_weights'])
        np.savez_compressed(os.path.join(OUT_M, run_id + '.opt.npz'),
                            **{k: np.asarray(v) for k, v in ow.items()})
    return mc, sum(int(np.prod(a.shape)) for a in w.values())


def main():
    only_missing = '--only-missing' in sys.argv
    os.makedirs(OUT_M, exist_ok=True)
    os.makedirs(OUT_D, exist_ok=True)
    files = sorted(glob.glob(REF + '/Model-*/Trained-Models-*/*.h5'))
    by_sig = {}
    for p in files:
        f = h5py.File(p, 'r')
        sig = signature(json.loads(f.attrs['model_config']))
        sz = os.path.getsize(p)
        if sig not in by_sig or sz < by_sig[sig][0]:
            by_sig[sig] = (sz, p)
    # exemplars above MAX_BYTES are skipped to keep the fixture set small (reported in index.json)
    chosen = {os.path.splitext(os.path.basename(p))[0]: p for sz, p in by_sig.values()
              if sz <= MAX_BYTES}
    skipped = sorted(os.path.relpath(p, REF) for sz, p in by_sig.values() if sz > MAX_BYTES)
    for p in files:
        rid = os.path.splitext(os.path.basename(p))[0]
        if rid in NAMED:
            chosen[rid] = p
    # the fused BlazeFace + both heads graph that blazeFaceDetectorH5.py:102 loads (config 5)
    for u in UNIFIED:
        chosen[u] = REF + '/BlazePoser/UnifiedModels/%s.h5' % u
    index = {}
    for rid, p in sorted(chosen.items()):
        key = rid
        if rid in index:  # same run id in two directories: keep directory prefix
            key = os.path.basename(os.path.dirname(p)) + '__' + rid
        if only_missing and os.path.exists(os.path.join(OUT_M, key + '.npz')):
            f = h5py.File(p, 'r')
            mc = strip(json.loads(f.attrs['model_config']))
            n = sum(int(np.prod(v.shape)) for v in np.load(os.path.join(OUT_M, key + '.npz')).values())
        else:
            mc, n = convert(p, key)
        sig = signature(mc)
        index[key] = {'dir': os.path.relpath(os.path.dirname(p), REF), 'n_params': n,
                      'signature_id': sorted(by_sig).index(sig) if sig in by_sig else -1}
    with open(os.path.join(OUT_M, 'index.json'), 'w') as fh:
        json.dump({'models': index, 'skipped_large_signatures': skipped}, fh, indent=1,
                  sort_keys=True)
    for d in DATASETS:
        if only_missing and os.path.exists(os.path.join(OUT_D, d)):
            continue
        shutil.copyfile(os.path.join(REF, 'FeatureMaps-Datasets', d), os.path.join(OUT_D, d))
    print('converted', len(index), 'checkpoints;', len(by_sig), 'signatures;',
          len(skipped), 'large signatures skipped')


if __name__ == '__main__':
    sys.exit(main())
