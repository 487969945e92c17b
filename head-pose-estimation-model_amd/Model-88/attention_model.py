"""Model-88/attention_model.py builders on the hpe Keras-compatible API.

se_transformer_regr_head (:16-80): SE channel gate (GAP -> Dense relu -> Dense sigmoid -> Multiply),
spatial multi-head self-attention over H*W tokens + residual + LayerNorm, FFN + residual +
LayerNorm, 1x1-conv head.  create_modelC (:82-95): SE gate + 1x1 head.  create_model_complex
(:97-169): 1x1 projection, three residual blocks of two softsign 1x1 convs, bottleneck, head.
On the reference's 1x1 feature maps every block is row-local and runs in the fused row program.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpe import keras  # noqa: E402
from hpe.keras import layers as kl  # noqa: E402


def _flatten_hw(t):          # Lambda bodies of attention_model.py:43-50 / :66-72; row-local
    return t


def _reshape_back(ts):
    return ts[0]


def se_transformer_regr_head(input_channels=88, reduction=16, num_heads=4, key_dim=16, ff_dim=64,
                             hidden_channels=128):
    x_in = kl.Input(shape=(None, None, input_channels))
    se = kl.GlobalAveragePooling2D()(x_in)
    se = kl.Dense(input_channels // reduction, activation='relu')(se)
    se = kl.Dense(input_channels, activation='sigmoid')(se)
    se = kl.Reshape((1, 1, input_channels))(se)
    gated = kl.Multiply()([x_in, se])
    flat = kl.Lambda(_flatten_hw)(gated)
    attn = kl.MultiHeadAttention(num_heads=num_heads, key_dim=key_dim)(flat, flat)
    h = kl.LayerNormalization()(kl.Add()([flat, attn]))
    ff = kl.Dense(input_channels)(kl.Dense(ff_dim, activation='relu')(h))
    h = kl.LayerNormalization()(kl.Add()([h, ff]))
    back = kl.Lambda(_reshape_back)([h, x_in])
    head = kl.Conv2D(hidden_channels, kernel_size=1, activation='relu')(back)
    out = kl.Conv2D(3, kernel_size=1, activation=None)(head)
    return keras.Model(inputs=x_in, outputs=out, name='SE_Transformer_Regr')


def create_modelC():
    inp = keras.Input((None, None, 88))
    se = kl.GlobalAveragePooling2D()(inp)
    se = kl.Dense(11, activation='relu')(se)
    se = kl.Dense(88, activation='sigmoid')(se)
    gated = kl.Multiply()([inp, kl.Reshape((1, 1, 88))(se)])
    h = kl.Conv2D(42, 1, activation='relu')(gated)
    return keras.Model(inp, kl.Conv2D(3, 1, activation=None)(h))


def create_model_complex(reg, dr):
    l2 = keras.regularizers.l2(reg)

    def conv(units, act, x):
        y = kl.Conv2D(filters=units, kernel_size=1, padding='same', activation=act,
                      kernel_regularizer=l2, kernel_initializer='glorot_uniform')(x)
        return y

    def res_block(inp, filters=16):
        y = kl.SpatialDropout2D(dr)(conv(filters, 'softsign', inp))
        y = kl.SpatialDropout2D(dr)(conv(filters, 'softsign', y))
        return kl.Activation('relu')(kl.Add()([inp, y]))

    inputs = keras.Input(shape=(None, None, 88))
    x = kl.SpatialDropout2D(dr)(conv(16, 'softsign', inputs))
    for _ in range(3):
        x = res_block(x, 16)
    x = kl.SpatialDropout2D(dr)(conv(8, 'softsign', x))
    outputs = conv(3, None, x)
    return keras.Model(inputs=inputs, outputs=outputs, name='Complex_Conv_Skip_Model')
