"""The helpers both reference drivers import from their own ``utilities.py`` (one implementation
here for Model-96/utilities.py and Model-88/utilities.py; line numbers below are Model-96's):
WandbCallback (:7-29), load_dataset (:31-34, in hpe.data), load_model_from_json (:36-41),
load_dataset_with_weights (:43-77), analyze_angle_distributions (:80-124; histogram counts are logged
instead of matplotlib images)."""
import numpy as np

from . import keras, runlog
from .data import load_dataset  # noqa: F401


class WandbCallback(keras.callbacks.Callback):
    def __init__(self):
        super().__init__()
        self.losses, self.val_losses, self.maes, self.val_maes = [], [], [], []

    def on_epoch_end(self, epoch, logs=None):
        self.losses.append(logs['loss'])
        self.val_losses.append(logs['val_loss'])
        self.maes.append(logs['mae'])
        self.val_maes.append(logs['val_mae'])
        runlog.log({'epoch': epoch, 'train_loss': logs['loss'], 'val_loss': logs['val_loss'],
                    'train_mae': logs['mae'], 'val_mae': logs['val_mae']})


def load_model_from_json(model_path):
    """Load a model architecture from a Keras JSON file (weights freshly initialised)."""
    import json
    with open(model_path) as f:
        cfg = json.load(f)
    return _model_from_json_config(cfg)


def _model_from_json_config(cfg):
    """Rebuild the Keras layer objects from a model_config so weights get Keras initialisers."""
    from hpe import layers as L
    from hpe.model import Model
    mc = cfg.get('config', cfg)
    tensors = {}
    for l in mc['layers']:
        c = dict(l['config'])
        cls = l['class_name']
        if cls == 'InputLayer':
            tensors[l['name']] = L.Input(shape=c['batch_input_shape'][1:], name=l['name'])
            continue
        ins = [tensors[t[0]] for node in l['inbound_nodes'] for t in node]
        kw = {k: c[k] for k in c if k not in ('name', 'trainable', 'dtype', 'kernel_initializer',
                                               'bias_initializer', 'activity_regularizer',
                                               'kernel_constraint', 'bias_constraint',
                                               'data_format', 'groups', 'noise_shape', 'seed',
                                               'registered_name')}
        for rk in ('kernel_regularizer', 'bias_regularizer'):
            if kw.get(rk):
                kw[rk] = L.l2(kw[rk]['config'].get('l2', 0.0))
        layer = getattr(L, cls)(name=l['name'], **kw)
        tensors[l['name']] = layer(ins if len(ins) > 1 else ins[0])
    return Model(tensors[mc['input_layers'][0][0]], tensors[mc['output_layers'][0][0]],
                 name=mc.get('name'))


def load_dataset_with_weights(npz_path):
    """Per-sample weights from the head off-axis angle (reference :43-77, Eq. 12-13)."""
    data = np.load(npz_path)
    features, poses = data['features'], data['poses']
    yaw_rad, pitch_rad = np.deg2rad(poses[:, 0]), np.deg2rad(poses[:, 1])
    cos_prod = np.clip(np.cos(pitch_rad) * np.cos(yaw_rad), -1.0, 1.0)
    delta_deg = np.rad2deg(np.arccos(cos_prod))
    weights = np.ones_like(delta_deg)
    mask = delta_deg > 60.0
    weights[mask] = 0.5 ** ((delta_deg[mask] - 60.0) / 5.0)
    return {'features': features, 'poses': poses, 'weights': weights}


def analyze_angle_distributions(train_poses, test_poses):
    """Histogram counts of yaw/pitch/roll for unique train / test poses (logged, not plotted)."""
    out = {}
    for name, arr in (('train', np.unique(train_poses.reshape(-1, 3), axis=0)),
                      ('test', np.unique(test_poses.reshape(-1, 3), axis=0))):
        for i, a in enumerate(('yaw', 'pitch', 'roll')):
            h, e = np.histogram(arr[:, i], bins=50)
            out['%s_%s_hist' % (name, a)] = h.tolist()
            out['%s_%s_edges' % (name, a)] = e.tolist()
    runlog.log({'angle_distributions': out})
    return out
