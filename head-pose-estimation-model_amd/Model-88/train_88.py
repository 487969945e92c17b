"""Model-88 training driver on the MI355X hot path (drop-in for Model-88/train_88.py).

Same ``config`` keys and defaults (train_88.py:45-64: SGD lr 2.8e-4, batch 128, dropout 1e-4,
l2 1e-6, 64 filters), the same builders (create_model :66-158, create_model_skip_fc :163-223,
bestmodelV1 :226-253, and create_model_complex from attention_model.py used by train() :309),
and the same train() flow (:256-397): BIWI_Train + BIWI_NoTrack enlarged sets concatenated,
angle-distribution analysis, reshape to (N,1,1,88), 80/20 split (random_state 42), compile,
ModelCheckpoint to Trained-Models-88/<run id>.h5, EarlyStopping, fit, evaluate on BIWI test and
AFLW2000.  Env FEATUREMAPS_DIR_PATH names the dataset directory.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

import hpe  # noqa: E402
from hpe import keras, runlog  # noqa: E402
from hpe.data import train_test_split  # noqa: E402
from attention_model import create_model_complex, create_modelC, se_transformer_regr_head  # noqa: E402,F401
from utilities import WandbCallback, analyze_angle_distributions, load_dataset  # noqa: E402

config = {
    'learning_rate': 0.00028,
    'batch_size': 128,
    'total_epochs': 1000000,
    'early_stopping_patience': 40,
    'early_stopping_min_delta': 0.001,
    'optimizer': 'sgd',
    'loss_function': 'mse',
    'performance_metrics': ['mae'],
    'save_best_only': True,
    'monitor_metric': 'val_loss',
    'dropout_rate': 0.0001,
    'filtersnum': 64,
    'regularizer_rate': 1e-6,
}


def _conv(units, act, reg, x):
    return keras.layers.Conv2D(filters=units, kernel_size=1, padding='same', activation=act,
                               kernel_initializer=keras.initializers.GlorotUniform(),
                               kernel_regularizer=reg)(x)


def create_model():
    """88 -> filtersnum softsign -> SpatialDropout -> 3 linear -> SpatialDropout (L2 on kernels)."""
    reg = keras.regularizers.l2(config['regularizer_rate'])
    inputs = keras.Input(shape=(None, None, 88))
    x0 = keras.layers.SpatialDropout2D(config['dropout_rate'])(
        _conv(config['filtersnum'], 'softsign', reg, inputs))
    x5 = keras.layers.SpatialDropout2D(config['dropout_rate'])(_conv(3, 'linear', reg, x0))
    return keras.Model(inputs=inputs, outputs=x5)


def create_model_skip_fc():
    """88 -> 32 -> 64 -> 32 (+ skip from the first block) -> 3, softsign, SpatialDropout, L2."""
    reg = keras.regularizers.l2(config['regularizer_rate'])
    dr = config['dropout_rate']
    inputs = keras.Input(shape=(None, None, 88))
    x1 = keras.layers.SpatialDropout2D(dr)(_conv(32, 'softsign', reg, inputs))
    x2 = keras.layers.SpatialDropout2D(dr)(_conv(64, 'softsign', reg, x1))
    x3 = keras.layers.Add()([_conv(32, 'softsign', reg, x2), x1])
    x3 = keras.layers.SpatialDropout2D(dr)(x3)
    outputs = _conv(3, 'linear', reg, x3)
    return keras.Model(inputs=inputs, outputs=outputs, name='FC_Skip_Regressor')


def bestmodelV1():
    reg = keras.regularizers.l2(config['regularizer_rate'])
    inputs = keras.Input(shape=(None, None, 88))
    x1 = keras.layers.SpatialDropout2D(config['dropout_rate'])(
        _conv(config['filtersnum'], 'softsign', reg, inputs))
    x2 = keras.layers.SpatialDropout2D(config['dropout_rate'])(_conv(3, 'linear', reg, x1))
    return keras.Model(inputs=inputs, outputs=x2)


def _optimizer():
    if config['optimizer'] == 'sgd':
        return keras.optimizers.SGD(learning_rate=config['learning_rate'])
    return keras.optimizers.Adam(learning_rate=config['learning_rate'])


def train(builder=None):
    run = runlog.init(project='HeadPoseRegressor-88features', config=config, notes='',
                      tags=['BIWI_Train+BIWI_NoTrack'])
    print('Loading datasets...')
    d = os.getenv('FEATUREMAPS_DIR_PATH', '')
    a_x, a_y = load_dataset(d + 'BIWI_Train_Enlarged_features_88_0.7_1.npz')
    b_x, b_y = load_dataset(d + 'BIWI_NoTrack_Enlarged_features_88_0.7_1.npz')
    tr_x, tr_y = np.concatenate((a_x, b_x), axis=0), np.concatenate((a_y, b_y), axis=0)
    te_x, te_y = load_dataset(d + 'BIWI_Test_Enlarged_features_88_0.7_1.npz')
    af_x, af_y = load_dataset(d + 'AFLW2000_Enlarged_features_88_0.7_1.npz')
    print(f'train_features shape: {tr_x.shape}')
    print(f'train_poses shape: {tr_y.shape}')
    analyze_angle_distributions(tr_y, te_y)
    tr_x, te_x, af_x = (a.reshape(-1, 1, 1, 88) for a in (tr_x, te_x, af_x))
    tr_y, te_y, af_y = (a.reshape(-1, 1, 1, 3) for a in (tr_y, te_y, af_y))
    tr_x, va_x, tr_y, va_y = train_test_split(tr_x, tr_y, test_size=0.2, random_state=42)
    model = (builder or (lambda: create_model_complex(config['regularizer_rate'],
                                                       config['dropout_rate'])))()
    model.compile(optimizer=_optimizer(), loss=config['loss_function'],
                  metrics=config['performance_metrics'])
    callbacks = [
        keras.callbacks.ModelCheckpoint(f'Trained-Models-88/{run.id}.h5',
                                        monitor=config['monitor_metric'],
                                        save_best_only=config['save_best_only']),
        keras.callbacks.EarlyStopping(monitor=config['monitor_metric'],
                                      patience=config['early_stopping_patience'],
                                      min_delta=config['early_stopping_min_delta'],
                                      restore_best_weights=True),
        WandbCallback(),
    ]
    history = model.fit(tr_x, tr_y, epochs=config['total_epochs'], batch_size=config['batch_size'],
                        validation_data=(va_x, va_y), callbacks=callbacks, verbose=1)
    tl, tm = model.evaluate(te_x, te_y, verbose=2)
    al, am = model.evaluate(af_x, af_y, verbose=2)
    print(f'Test loss on AFLW2000: {al}')
    print(f'Test MAE on AFLW2000: {am}')
    print(f'Test loss on BIWI_Test: {tl}')
    print(f'Test MAE on BIWI_Test: {tm}')
    run.summary.update({'test_loss': tl, 'test_mae': tm, 'test_loss_AFLW2000': al,
                        'test_mae_AFLW2000': am, 'total_parameters': model.count_params(),
                        'model_architecture': model.to_json()})
    best = int(np.argmin(history.history['val_loss']))
    runlog.log({'best_epoch': best + 1, 'best_epoch_train_loss': history.history['loss'][best],
                'best_epoch_train_mae': history.history['mae'][best],
                'best_epoch_val_loss': history.history['val_loss'][best],
                'best_epoch_val_mae': history.history['val_mae'][best]})
    run.finish()
    return model, history


if __name__ == '__main__':
    train()
