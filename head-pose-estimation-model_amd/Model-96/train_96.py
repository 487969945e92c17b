"""Model-96 training driver on the MI355X hot path (drop-in for Model-96/train_96.py).

Same entry point and contract: ``python train_96.py --dropout_rate D --regularizer_rate R
--num_filters F``; env FEATUREMAPS_DIR_PATH (dataset directory) and
TRAINED_MODELS_96_RESHAPEDINPUT_NOFLATTEN_PATH (checkpoint directory); the module-level ``config``
dict with the reference's keys and -1 sentinels (train_96.py:42-59), so omitting a flag still
fails inside the model builder; create_model() builds the same graph (:65-110); train() follows
the same data flow (:113-209): load, reshape to (N,1,1,96), 80/20 split with random_state 42,
ModelCheckpoint(save_best_only) + EarlyStopping(restore_best_weights) + the wandb-style logger,
fit, evaluate on BIWI test and AFLW2000.  Tensor math runs in libhpe.so (HIP, gfx950).
"""
import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

import hpe  # noqa: E402
from hpe import keras, runlog  # noqa: E402
from hpe.data import train_test_split  # noqa: E402
from utilities import WandbCallback, load_dataset  # noqa: E402

RANDOM_SEED = 42
np.random.seed(RANDOM_SEED)
hpe.set_seed(RANDOM_SEED)

config = {
    'learning_rate': 0.00028,
    'batch_size': 128,
    'total_epochs': 10000,
    'early_stopping_patience': 40,
    'early_stopping_min_delta': 0.001,
    'optimizer': 'adam',
    'loss_function': 'mse',
    'performance_metrics': ['mae'],
    'save_best_only': True,
    'monitor_metric': 'val_loss',
    'dropout_rate': -1,
    'regularizer_rate': -1,
    'num_filters': -1,
}


def _optimizer():
    lr = config['learning_rate']
    name = config['optimizer']
    if name == 'adamax':
        return keras.optimizers.Adamax(learning_rate=lr)
    if name == 'sgd':
        return keras.optimizers.SGD(learning_rate=lr)
    return keras.optimizers.Adam(learning_rate=lr)


def create_model():
    """96 -> num_filters (1x1 conv, tanh) -> SpatialDropout -> 3 (1x1 conv) -> SpatialDropout,
    L2 on kernels and biases; compiled with mse / mae."""
    reg = keras.regularizers.l2(config['regularizer_rate'])

    def conv(units, act):
        return keras.layers.Conv2D(filters=units, kernel_size=1, padding='same', activation=act,
                                   kernel_initializer=keras.initializers.GlorotUniform(),
                                   kernel_regularizer=reg, bias_regularizer=reg)

    inputs = keras.Input(shape=(None, None, 96))
    h = keras.layers.SpatialDropout2D(config['dropout_rate'])(conv(config['num_filters'], 'tanh')(inputs))
    out = keras.layers.SpatialDropout2D(config['dropout_rate'])(conv(3, None)(h))
    model = keras.Model(inputs=inputs, outputs=out)
    model.compile(optimizer=_optimizer(), loss=config['loss_function'],
                  metrics=config['performance_metrics'])
    return model


def _as_maps(a, c):
    return np.asarray(a).reshape(-1, 1, 1, c)


def train():
    run = runlog.init(project='HeadPoseRegressor-BIWI-96features', config=config, notes='',
                      tags=['BIWI_Train'])
    data_dir = os.getenv('FEATUREMAPS_DIR_PATH', '')
    print('Loading datasets...')
    # the reference joins the first path without a separator (train_96.py:124) and the others with
    # one (:128,130); both are kept
    tr_x, tr_y = load_dataset(f'{data_dir}BIWI_train_features_96.npz')
    te_x, te_y = load_dataset(f'{data_dir}/BIWI_test_features_96.npz')
    af_x, af_y = load_dataset(f'{data_dir}/AFLW2000_features_96_0.7_1.npz')
    tr_x, te_x, af_x = _as_maps(tr_x, 96), _as_maps(te_x, 96), _as_maps(af_x, 96)
    tr_y, te_y, af_y = _as_maps(tr_y, 3), _as_maps(te_y, 3), _as_maps(af_y, 3)
    tr_x, va_x, tr_y, va_y = train_test_split(tr_x, tr_y, test_size=0.2, random_state=42)
    ckpt_dir = os.getenv('TRAINED_MODELS_96_RESHAPEDINPUT_NOFLATTEN_PATH', '.')
    callbacks = [
        keras.callbacks.ModelCheckpoint(f'{ckpt_dir}/{run.id}.h5', monitor=config['monitor_metric'],
                                        save_best_only=config['save_best_only']),
        keras.callbacks.EarlyStopping(monitor=config['monitor_metric'],
                                      patience=config['early_stopping_patience'],
                                      min_delta=config['early_stopping_min_delta'],
                                      restore_best_weights=True),
        WandbCallback(),
    ]
    model = create_model()
    history = model.fit(tr_x, tr_y, epochs=config['total_epochs'], batch_size=config['batch_size'],
                        validation_data=(va_x, va_y), callbacks=callbacks, verbose=1)
    test_loss, test_mae = model.evaluate(te_x, te_y, verbose=2)
    af_loss, af_mae = model.evaluate(af_x, af_y, verbose=2)
    run.summary.update({'test_AFLW2000_mae': af_mae, 'test_AFLW2000_loss': af_loss,
                        'test_loss': test_loss, 'test_mae': test_mae,
                        'total_parameters': model.count_params(),
                        'model_architecture': model.to_json()})
    best = int(np.argmin(history.history['val_loss']))
    runlog.log({'best_epoch': best + 1,
                'best_epoch_train_loss': history.history['loss'][best],
                'best_epoch_train_mae': history.history['mae'][best],
                'best_epoch_val_loss': history.history['val_loss'][best],
                'best_epoch_val_mae': history.history['val_mae'][best]})
    run.finish()
    return model, history


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--dropout_rate', type=float, default=config['dropout_rate'])
    ap.add_argument('--regularizer_rate', type=float, default=config['regularizer_rate'])
    ap.add_argument('--num_filters', type=int, default=config['num_filters'])
    config.update(vars(ap.parse_args(argv)))
    return train()


if __name__ == '__main__':
    main()
