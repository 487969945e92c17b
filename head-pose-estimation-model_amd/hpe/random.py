"""Seeded host RNG for weight initialisation, fit() shuffling and the dropout seed stream.

TF's RNG streams cannot be reproduced (SURVEY.md §7 hard part iii); ``set_seed`` plays the role of
``np.random.seed / tf.random.set_seed`` in train_96.py:20-23 for this implementation."""
import numpy as np

_state = {'seed': 42, 'gen': np.random.default_rng(42)}


def set_seed(seed):
    _state['seed'] = int(seed)
    _state['gen'] = np.random.default_rng(int(seed))


def generator():
    return _state['gen']


def seed():
    return _state['seed']


def dropout_seed(iteration):
    """Dropout hash seed of optimizer step ``iteration`` (1-based) in fit()."""
    return (_state['seed'] * 1000003 + int(iteration)) & 0xFFFFFFFFFFFFFFFF
