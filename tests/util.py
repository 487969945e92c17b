"""Shared helpers for the parity tests (fixtures, synthetic inputs, oracle glue)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')
MODELS = os.path.join(GOLDEN, 'models')
DATA = os.path.join(GOLDEN, 'data')

# forward tolerance: the reference's own rtol (InputShapeConvertor.py:205) with
# atol widened to 1e-4 degrees for accumulation-order differences
RTOL, ATOL = 1e-5, 1e-4


def index():
    with open(os.path.join(MODELS, 'index.json')) as fh:
        return json.load(fh)['models']


def fixture(rid):
    with open(os.path.join(MODELS, rid + '.json')) as fh:
        meta = json.load(fh)
    w = dict(np.load(os.path.join(MODELS, rid + '.npz')))
    return meta['model_config'], w


def input_channels(mc):
    return mc['config']['layers'][0]['config']['batch_input_shape'][-1]


def features(n, c, seed=0, h=1, w=1):
    """Synthetic post-ReLU-like BlazeFace features: max(0, 0.6 N(0,1) - 0.3)."""
    rng = np.random.default_rng(seed)
    return np.maximum(0.0, 0.6 * rng.standard_normal((n, h, w, c)) - 0.3).astype(np.float32)


def labels(n, seed=1):
    return (20.0 * np.random.default_rng(seed).standard_normal((n, 3))).astype(np.float32)
