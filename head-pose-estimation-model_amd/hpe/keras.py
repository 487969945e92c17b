"""``keras``-shaped namespace so the reference's builder code reads unchanged:

    from hpe import keras
    x = keras.layers.Conv2D(filters=360, kernel_size=1, activation='tanh',
                            kernel_regularizer=keras.regularizers.l2(0.1))(keras.Input((None, None, 96)))
"""
import types

from . import callbacks as _cb
from . import layers as _L
from . import model as _M
from . import optimizers as _O
from . import random as _R

layers = types.SimpleNamespace(
    Input=_L.Input, InputLayer=_L.InputLayer, Conv2D=_L.Conv2D, Dense=_L.Dense,
    SeparableConv2D=_L.SeparableConv2D, SpatialDropout2D=_L.SpatialDropout2D,
    Dropout=_L.Dropout, Activation=_L.Activation, ReLU=_L.ReLU, Add=_L.Add, Average=_L.Average,
    Multiply=_L.Multiply, Flatten=_L.Flatten, Reshape=_L.Reshape,
    GlobalAveragePooling2D=_L.GlobalAveragePooling2D, Lambda=_L.Lambda,
    LayerNormalization=_L.LayerNormalization, BatchNormalization=_L.BatchNormalization,
    MultiHeadAttention=_L.MultiHeadAttention)
regularizers = types.SimpleNamespace(l2=_L.l2, L2=_L.L2)
initializers = types.SimpleNamespace(GlorotUniform=_L.GlorotUniform, Zeros=_L.Zeros, Ones=_L.Ones)
optimizers = types.SimpleNamespace(SGD=_O.SGD, Adam=_O.Adam, Adamax=_O.Adamax,
                                   legacy=types.SimpleNamespace(SGD=_O.SGD, Adam=_O.Adam,
                                                                Adamax=_O.Adamax))
callbacks = types.SimpleNamespace(Callback=_cb.Callback, History=_cb.History,
                                  ModelCheckpoint=_cb.ModelCheckpoint,
                                  EarlyStopping=_cb.EarlyStopping)
models = types.SimpleNamespace(load_model=_M.load_model, model_from_config=_M.model_from_config)
backend = types.SimpleNamespace(clear_session=_L.clear_session)
utils = types.SimpleNamespace(set_random_seed=_R.set_seed)
Input = _L.Input
Model = _M.Model
