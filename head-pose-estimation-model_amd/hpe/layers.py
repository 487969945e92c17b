"""Keras-compatible functional layer API for the head-pose regressors.

Mirrors the ``keras.layers`` surface the reference builds its models with
(Model-96/train_96.py:65-110, Model-88/train_88.py:66-253, Model-88/attention_model.py:1-169):
same class names, constructor arguments, auto-naming (``conv2d``, ``conv2d_1`` ...), argument
validation errors (ValueError), and the same serialised ``model_config`` JSON a Keras 2.13 ``.h5``
stores -- which is what hpe/compiler.py lowers to the HIP row program.  Layers here only describe
the graph and create initial weights; all arithmetic runs in libhpe.so.
"""
import collections
import math
import re

import numpy as np

from . import random as hrandom

_NAME_COUNTS = collections.defaultdict(int)


def clear_session():
    _NAME_COUNTS.clear()


def _snake(name):
    s = re.sub(r'(.)([A-Z][a-z0-9]+)', r'\1_\2', name)
    s = re.sub(r'([a-z])([A-Z])', r'\1_\2', s).lower()
    return s.replace('2_d', '2d').replace('1_d', '1d')


def unique_name(base, zero_based=True):
    n = _NAME_COUNTS[base]
    _NAME_COUNTS[base] += 1
    if zero_based:
        return base if n == 0 else '%s_%d' % (base, n)
    return '%s_%d' % (base, n + 1)


# ----------------------------------------------------------------------------------------------
# regularizers / initializers (keras.regularizers.l2, keras.initializers.GlorotUniform)
# ----------------------------------------------------------------------------------------------
class L2:
    def __init__(self, l2=0.01):
        if not isinstance(l2, (int, float, np.floating)) or math.isinf(l2) or math.isnan(l2):
            raise ValueError('Value of `l2` must be a finite number. Received: l2=%r' % (l2,))
        self.l2 = float(l2)

    def get_config(self):
        return {'l2': float(np.float32(self.l2))}

    def serialize(self):
        return {'module': 'keras.regularizers', 'class_name': 'L2', 'config': self.get_config(),
                'registered_name': None}

    def __call__(self, x):
        return self.l2 * float(np.sum(np.square(x)))


def l2(l2=0.01):
    return L2(l2)


def _ser_reg(r):
    if r is None:
        return None
    if isinstance(r, L2):
        return r.serialize()
    if isinstance(r, dict):
        return r
    raise ValueError('unsupported regularizer %r' % (r,))


def _fans(shape):
    if len(shape) < 1:
        return 1, 1
    if len(shape) == 1:
        return shape[0], shape[0]
    if len(shape) == 2:
        return shape[0], shape[1]
    rf = int(np.prod(shape[:-2]))
    return shape[-2] * rf, shape[-1] * rf


class GlorotUniform:
    def __init__(self, seed=None):
        self.seed = seed

    def __call__(self, shape):
        fi, fo = _fans(shape)
        limit = math.sqrt(6.0 / max(1.0, (fi + fo)))
        rng = np.random.default_rng(self.seed) if self.seed is not None else hrandom.generator()
        return rng.uniform(-limit, limit, size=shape).astype(np.float32)

    def serialize(self):
        return {'module': 'keras.initializers', 'class_name': 'GlorotUniform',
                'config': {'seed': self.seed}, 'registered_name': None}


class Zeros:
    def __call__(self, shape):
        return np.zeros(shape, dtype=np.float32)

    def serialize(self):
        return {'module': 'keras.initializers', 'class_name': 'Zeros', 'config': {},
                'registered_name': None}


class Ones(Zeros):
    def __call__(self, shape):
        return np.ones(shape, dtype=np.float32)

    def serialize(self):
        return {'module': 'keras.initializers', 'class_name': 'Ones', 'config': {},
                'registered_name': None}


def get_initializer(x):
    if x is None or x == 'glorot_uniform':
        return GlorotUniform()
    if x == 'zeros':
        return Zeros()
    if x == 'ones':
        return Ones()
    if hasattr(x, '__call__') and hasattr(x, 'serialize'):
        return x
    raise ValueError('Unknown initializer: %r' % (x,))


_ACTIVATIONS = ('linear', 'tanh', 'relu', 'softsign', 'sigmoid', 'elu', 'selu', 'swish',
                'softplus', 'leaky_relu')


def _act(a):
    if a is None:
        return 'linear'
    if a not in _ACTIVATIONS:
        raise ValueError('Unknown activation function: %r' % (a,))
    return a


# ----------------------------------------------------------------------------------------------
# graph nodes
# ----------------------------------------------------------------------------------------------
class KerasTensor:
    def __init__(self, shape, layer, index=0):
        self.shape = tuple(shape)   # without batch
        self.layer = layer
        self.index = index

    def __repr__(self):
        return 'KerasTensor(shape=%s, layer=%s)' % ((None,) + self.shape, self.layer.name)


class Layer:
    zero_based = True

    def __init__(self, name=None, trainable=True, dtype='float32', **kwargs):
        base = _snake(type(self).__name__)
        self.name = name if name else unique_name(base, self.zero_based)
        self.trainable = trainable
        self.dtype = dtype
        self.inbound = None
        self.inbound_kw = {}
        self.output = None
        self.weights = collections.OrderedDict()   # relative key -> array

    # -- to override ---------------------------------------------------------------------------
    def output_shape(self, shapes):
        return shapes[0]

    def build(self, shapes):
        pass

    def layer_config(self):
        return {}

    # -------------------------------------------------------------------------------------------
    def get_config(self):
        c = {'name': self.name, 'trainable': self.trainable, 'dtype': self.dtype}
        c.update(self.layer_config())
        return c

    def __call__(self, inputs, *args, **kwargs):
        if self.inbound is not None:
            raise ValueError('layer %s is already connected (shared layers are not supported)'
                             % self.name)
        ins = list(inputs) if isinstance(inputs, (list, tuple)) else [inputs]
        ins += [a for a in args if isinstance(a, KerasTensor)]
        for t in ins:
            if not isinstance(t, KerasTensor):
                raise ValueError('%s expects KerasTensor inputs, got %r' % (self.name, type(t)))
        self.inbound = ins
        self.inbound_kw = {k: v for k, v in kwargs.items() if isinstance(v, KerasTensor)}
        shapes = [t.shape for t in ins]
        self.build(shapes)
        self.output = KerasTensor(self.output_shape(shapes), self)
        return self.output

    def count_params(self):
        return int(sum(int(np.prod(w.shape)) for w in self.weights.values()))


class InputLayer(Layer):
    zero_based = False

    def __init__(self, shape, name=None, **kw):
        super().__init__(name=name if name else unique_name('input', False), **kw)
        self.shape = tuple(shape)
        self.output = KerasTensor(self.shape, self)
        self.inbound = []

    def get_config(self):
        return {'batch_input_shape': [None] + list(self.shape), 'dtype': 'float32',
                'sparse': False, 'ragged': False, 'name': self.name}


def Input(shape=None, name=None, batch_size=None, **kw):
    return InputLayer(shape, name=name).output


def _check_positive(v, what):
    if not isinstance(v, (int, np.integer)) or isinstance(v, bool):
        if isinstance(v, float) and v.is_integer() and v > 0:
            return int(v)
        raise ValueError('Invalid value for argument `%s`. Expected a strictly positive value. '
                         'Received %s=%r.' % (what, what, v))
    if v <= 0:
        raise ValueError('Invalid value for argument `%s`. Expected a strictly positive value. '
                         'Received %s=%r.' % (what, what, v))
    return int(v)


def _pair(v):
    return [int(v), int(v)] if isinstance(v, (int, np.integer)) else [int(a) for a in v]


class Conv2D(Layer):
    def __init__(self, filters, kernel_size, strides=(1, 1), padding='valid',
                 data_format=None, dilation_rate=(1, 1), groups=1, activation=None,
                 use_bias=True, kernel_initializer='glorot_uniform', bias_initializer='zeros',
                 kernel_regularizer=None, bias_regularizer=None, activity_regularizer=None,
                 kernel_constraint=None, bias_constraint=None, **kw):
        super().__init__(**kw)
        self.filters = _check_positive(filters, 'filters')
        self.kernel_size = _pair(kernel_size)
        self.strides = _pair(strides)
        self.padding = padding.lower()
        if self.padding not in ('same', 'valid'):
            raise ValueError('padding must be same|valid')
        self.dilation_rate = _pair(dilation_rate)
        self.activation = _act(activation)
        self.use_bias = use_bias
        self.kinit = get_initializer(kernel_initializer)
        self.binit = get_initializer(bias_initializer)
        self.kreg, self.breg = kernel_regularizer, bias_regularizer

    def output_shape(self, shapes):
        return tuple(shapes[0][:-1]) + (self.filters,)

    def build(self, shapes):
        cin = shapes[0][-1]
        self.weights['kernel'] = self.kinit(tuple(self.kernel_size) + (cin, self.filters))
        if self.use_bias:
            self.weights['bias'] = self.binit((self.filters,))

    def layer_config(self):
        return {'filters': self.filters, 'kernel_size': self.kernel_size, 'strides': self.strides,
                'padding': self.padding, 'data_format': 'channels_last',
                'dilation_rate': self.dilation_rate, 'groups': 1, 'activation': self.activation,
                'use_bias': self.use_bias, 'kernel_initializer': self.kinit.serialize(),
                'bias_initializer': self.binit.serialize(),
                'kernel_regularizer': _ser_reg(self.kreg), 'bias_regularizer': _ser_reg(self.breg),
                'activity_regularizer': None, 'kernel_constraint': None, 'bias_constraint': None}


class Dense(Layer):
    def __init__(self, units, activation=None, use_bias=True, kernel_initializer='glorot_uniform',
                 bias_initializer='zeros', kernel_regularizer=None, bias_regularizer=None, **kw):
        super().__init__(**kw)
        self.units = _check_positive(units, 'units')
        self.activation = _act(activation)
        self.use_bias = use_bias
        self.kinit = get_initializer(kernel_initializer)
        self.binit = get_initializer(bias_initializer)
        self.kreg, self.breg = kernel_regularizer, bias_regularizer

    def output_shape(self, shapes):
        return tuple(shapes[0][:-1]) + (self.units,)

    def build(self, shapes):
        self.weights['kernel'] = self.kinit((shapes[0][-1], self.units))
        if self.use_bias:
            self.weights['bias'] = self.binit((self.units,))

    def layer_config(self):
        return {'units': self.units, 'activation': self.activation, 'use_bias': self.use_bias,
                'kernel_initializer': self.kinit.serialize(),
                'bias_initializer': self.binit.serialize(),
                'kernel_regularizer': _ser_reg(self.kreg), 'bias_regularizer': _ser_reg(self.breg),
                'activity_regularizer': None, 'kernel_constraint': None, 'bias_constraint': None}


class SeparableConv2D(Layer):
    def __init__(self, filters, kernel_size, strides=(1, 1), padding='valid', depth_multiplier=1,
                 activation=None, use_bias=True, depthwise_initializer='glorot_uniform',
                 pointwise_initializer='glorot_uniform', bias_initializer='zeros',
                 depthwise_regularizer=None, pointwise_regularizer=None, bias_regularizer=None, **kw):
        super().__init__(**kw)
        self.filters = _check_positive(filters, 'filters')
        self.kernel_size = _pair(kernel_size)
        self.strides = _pair(strides)
        self.padding = padding
        self.depth_multiplier = depth_multiplier
        self.activation = _act(activation)
        self.use_bias = use_bias
        self.dinit = get_initializer(depthwise_initializer)
        self.pinit = get_initializer(pointwise_initializer)
        self.binit = get_initializer(bias_initializer)
        self.dreg, self.preg, self.breg = depthwise_regularizer, pointwise_regularizer, bias_regularizer

    def output_shape(self, shapes):
        return tuple(shapes[0][:-1]) + (self.filters,)

    def build(self, shapes):
        cin = shapes[0][-1]
        self.weights['depthwise_kernel'] = self.dinit(tuple(self.kernel_size) + (cin, self.depth_multiplier))
        self.weights['pointwise_kernel'] = self.pinit((1, 1, cin * self.depth_multiplier, self.filters))
        if self.use_bias:
            self.weights['bias'] = self.binit((self.filters,))

    def layer_config(self):
        return {'filters': self.filters, 'kernel_size': self.kernel_size, 'strides': self.strides,
                'padding': self.padding, 'data_format': 'channels_last', 'dilation_rate': [1, 1],
                'groups': 1, 'activation': self.activation, 'use_bias': self.use_bias,
                'depth_multiplier': self.depth_multiplier,
                'depthwise_regularizer': _ser_reg(self.dreg),
                'pointwise_regularizer': _ser_reg(self.preg),
                'bias_regularizer': _ser_reg(self.breg), 'kernel_regularizer': None}


class SpatialDropout2D(Layer):
    def __init__(self, rate, data_format=None, **kw):
        super().__init__(**kw)
        if isinstance(rate, (int, float)) and not 0 <= rate <= 1:
            raise ValueError('Invalid value %s received for `rate`, expected a value between 0 '
                             'and 1.' % rate)
        self.rate = float(rate)

    def layer_config(self):
        return {'rate': self.rate, 'noise_shape': None, 'seed': None}


class Dropout(SpatialDropout2D):
    pass


class Activation(Layer):
    def __init__(self, activation, **kw):
        super().__init__(**kw)
        self.activation = _act(activation)

    def layer_config(self):
        return {'activation': self.activation}


class ReLU(Layer):
    def layer_config(self):
        return {'max_value': None, 'negative_slope': 0.0, 'threshold': 0.0}


class _Merge(Layer):
    def output_shape(self, shapes):
        return tuple(max(a, b) if a is not None and b is not None else (a or b)
                     for a, b in zip(*shapes[:2])) if len(shapes) > 1 else shapes[0]


class Add(_Merge):
    pass


class Average(_Merge):
    pass


class Multiply(_Merge):
    pass


class Flatten(Layer):
    def output_shape(self, shapes):
        s = shapes[0]
        if any(d is None for d in s):
            return (None,)
        return (int(np.prod(s)),)

    def layer_config(self):
        return {'data_format': 'channels_last'}


class Reshape(Layer):
    def __init__(self, target_shape, **kw):
        super().__init__(**kw)
        self.target_shape = tuple(target_shape)

    def output_shape(self, shapes):
        return self.target_shape

    def layer_config(self):
        return {'target_shape': list(self.target_shape)}


class GlobalAveragePooling2D(Layer):
    def __init__(self, data_format=None, keepdims=False, **kw):
        super().__init__(**kw)
        self.keepdims = keepdims

    def output_shape(self, shapes):
        c = shapes[0][-1]
        return (1, 1, c) if self.keepdims else (c,)

    def layer_config(self):
        return {'data_format': 'channels_last', 'keepdims': self.keepdims}


class Lambda(Layer):
    """Only the two reshape lambdas of attention_model.py:43-50,66-72 (row-local identities)."""

    def __init__(self, function, output_shape=None, **kw):
        super().__init__(**kw)
        self.function = function

    def output_shape(self, shapes):
        if len(shapes) == 2:
            return tuple(shapes[1][:-1]) + (shapes[0][-1],)
        s = shapes[0]
        return (None, s[-1])

    def layer_config(self):
        return {'function': getattr(self.function, '__name__', 'lambda'), 'function_type': 'lambda',
                'module': getattr(self.function, '__module__', None), 'output_shape': None,
                'arguments': {}}


class LayerNormalization(Layer):
    def __init__(self, axis=-1, epsilon=1e-3, center=True, scale=True, **kw):
        super().__init__(**kw)
        self.axis, self.epsilon, self.center, self.scale = axis, epsilon, center, scale

    def build(self, shapes):
        c = shapes[0][-1]
        self._axis = [len(shapes[0])]
        if self.scale:
            self.weights['gamma'] = np.ones((c,), np.float32)
        if self.center:
            self.weights['beta'] = np.zeros((c,), np.float32)

    def layer_config(self):
        return {'axis': getattr(self, '_axis', [-1]), 'epsilon': self.epsilon,
                'center': self.center, 'scale': self.scale}


class BatchNormalization(Layer):
    def __init__(self, axis=-1, momentum=0.99, epsilon=1e-3, center=True, scale=True, **kw):
        super().__init__(**kw)
        self.axis, self.momentum, self.epsilon, self.center, self.scale = axis, momentum, epsilon, center, scale

    def build(self, shapes):
        c = shapes[0][-1]
        if self.scale:
            self.weights['gamma'] = np.ones((c,), np.float32)
        if self.center:
            self.weights['beta'] = np.zeros((c,), np.float32)
        self.weights['moving_mean'] = np.zeros((c,), np.float32)
        self.weights['moving_variance'] = np.ones((c,), np.float32)

    def layer_config(self):
        return {'axis': [3], 'momentum': self.momentum, 'epsilon': self.epsilon,
                'center': self.center, 'scale': self.scale}


class MultiHeadAttention(Layer):
    def __init__(self, num_heads, key_dim, value_dim=None, dropout=0.0, use_bias=True,
                 output_shape=None, attention_axes=None, kernel_initializer='glorot_uniform',
                 bias_initializer='zeros', **kw):
        super().__init__(**kw)
        self.num_heads, self.key_dim = int(num_heads), int(key_dim)
        self.value_dim = int(value_dim) if value_dim else self.key_dim
        self.dropout, self.use_bias = dropout, use_bias
        self.kinit = get_initializer(kernel_initializer)
        self.binit = get_initializer(bias_initializer)

    def __call__(self, query, value=None, key=None, **kw):
        ins = [query]
        out = super().__call__(ins)
        if value is not None and value is not query:
            self.inbound_kw['value'] = value
        elif value is not None:
            self.inbound_kw['value'] = value
        if key is not None:
            self.inbound_kw['key'] = key
        return out

    def build(self, shapes):
        c = shapes[0][-1]
        h, d, dv = self.num_heads, self.key_dim, self.value_dim
        for part, dd in (('query', d), ('key', d), ('value', dv)):
            self.weights[part + '/kernel'] = self.kinit((c, h, dd))
            if self.use_bias:
                self.weights[part + '/bias'] = self.binit((h, dd))
        self.weights['attention_output/kernel'] = self.kinit((h, dv, c))
        if self.use_bias:
            self.weights['attention_output/bias'] = self.binit((c,))

    def layer_config(self):
        return {'num_heads': self.num_heads, 'key_dim': self.key_dim,
                'value_dim': self.value_dim, 'dropout': self.dropout, 'use_bias': self.use_bias,
                'output_shape': None, 'attention_axes': [1]}


# ----------------------------------------------------------------------------------------------
# functional graph -> Keras model_config
# ----------------------------------------------------------------------------------------------
def collect(inputs, outputs):
    """Layers reachable from outputs, in creation-consistent topological order."""
    seen, order = set(), []

    def visit(layer):
        if id(layer) in seen:
            return
        seen.add(id(layer))
        for t in (layer.inbound or []):
            visit(t.layer)
        for t in layer.inbound_kw.values():
            visit(t.layer)
        order.append(layer)
    for o in outputs:
        visit(o.layer)
    return order


def model_config(name, inputs, outputs):
    layers = collect(inputs, outputs)
    cfg_layers = []
    for l in layers:
        cls = 'InputLayer' if isinstance(l, InputLayer) else type(l).__name__
        nodes = []
        if l.inbound:
            kwmap = {}
            if l.inbound_kw:
                kwmap = {k: [t.layer.name, 0, 0] for k, t in l.inbound_kw.items()}
            node = [[t.layer.name, 0, 0, dict(kwmap) if i == 0 else {}]
                    for i, t in enumerate(l.inbound)]
            nodes = [node]
        cfg_layers.append({'class_name': cls, 'config': l.get_config(), 'name': l.name,
                           'inbound_nodes': nodes})
    return {'name': name, 'trainable': True, 'layers': cfg_layers,
            'input_layers': [[t.layer.name, 0, 0] for t in inputs],
            'output_layers': [[t.layer.name, 0, 0] for t in outputs]}, layers
