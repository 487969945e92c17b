"""Rewrite the committed reference checkpoints under tests/golden/h5/ with every Lambda layer's
marshalled Python bytecode replaced by '<bytecode stripped>' (reference bytecode must not
travel, in any form).  Uses the repo's own reader and Keras-2.13 legacy writer (hpe/h5io.py); the
weights, optimizer state and training_config are carried over unchanged.

    python tests/golden/strip_h5_bytecode.py          # rewrites files that still carry bytecode
"""
import glob
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, '..', '..', 'head-pose-estimation-model_amd'))
from hpe import h5io  # noqa: E402


def raw_model_config(path):
    f = h5io._File(path)
    return json.loads(h5io._txt(f.attrs(f.root)['model_config']))


def lambda_functions(mc):
    return [l['config'].get('function') for l in mc.get('config', {}).get('layers', [])
            if l.get('class_name') == 'Lambda']


def layer_weights(mc, w):
    out = []
    for l in mc['config']['layers']:
        ln = l['name']
        ws = [(k[len(ln) + 1:] + ':0' if l['class_name'] == 'Functional' else k + ':0', a)
              for k, a in w.items() if k.startswith(ln + '/')]
        out.append((ln, ws))
    return out


def strip(path):
    if all(f == '<bytecode stripped>' for f in lambda_functions(raw_model_config(path))):
        return False
    mc, w, opt = h5io.read_keras_h5(path, with_optimizer=True)   # the reader strips Lambda bytecode
    tc = h5io.read_training_config(path)
    tmp = path + '.tmp'
    h5io.write_keras_h5(tmp, mc, layer_weights(mc, w), tc, [(k + ':0', v) for k, v in opt.items()] or None)
    os.replace(tmp, path)
    return True


if __name__ == '__main__':
    for p in sorted(glob.glob(os.path.join(HERE, 'h5', '*.h5'))):
        print(p, 'rewritten' if strip(p) else 'clean')
