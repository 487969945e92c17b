"""keras.callbacks used by the reference's fit loop (Model-96/train_96.py:153-172,
Model-88/train_88.py:333-352): ModelCheckpoint(save_best_only), EarlyStopping(restore_best_weights),
plus History and the Callback base for WandbCallback-style subclasses (utilities.py:11-33)."""
import numpy as np


class Callback:
    def __init__(self):
        self.model = None
        self.params = {}

    def set_model(self, model):
        self.model = model

    def set_params(self, params):
        self.params = params

    def on_train_begin(self, logs=None):
        pass

    def on_train_end(self, logs=None):
        pass

    def on_epoch_begin(self, epoch, logs=None):
        pass

    def on_epoch_end(self, epoch, logs=None):
        pass


class History(Callback):
    def __init__(self):
        super().__init__()
        self.history = {}
        self.epoch = []

    def on_train_begin(self, logs=None):
        self.epoch = []

    def on_epoch_end(self, epoch, logs=None):
        self.epoch.append(epoch)
        for k, v in (logs or {}).items():
            self.history.setdefault(k, []).append(v)


class ModelCheckpoint(Callback):
    """Keras 2.13 semantics: mode 'auto' -> min for *loss*; save when current < best (no delta)."""

    def __init__(self, filepath, monitor='val_loss', verbose=0, save_best_only=False,
                 save_weights_only=False, mode='auto', **kw):
        super().__init__()
        self.filepath, self.monitor, self.verbose = filepath, monitor, verbose
        self.save_best_only, self.save_weights_only = save_best_only, save_weights_only
        if mode == 'max' or (mode == 'auto' and ('acc' in monitor or monitor.startswith('fmeasure'))):
            self.op, self.best = np.greater, -np.inf
        else:
            self.op, self.best = np.less, np.inf

    def on_epoch_end(self, epoch, logs=None):
        logs = logs or {}
        path = str(self.filepath).format(epoch=epoch + 1, **logs)
        if self.save_best_only:
            cur = logs.get(self.monitor)
            if cur is None:
                return
            if self.op(cur, self.best):
                if self.verbose:
                    print('\nEpoch %05d: %s improved from %.5f to %.5f, saving model to %s'
                          % (epoch + 1, self.monitor, self.best, cur, path))
                self.best = cur
                self.model.save(path)
        else:
            self.model.save(path)


class EarlyStopping(Callback):
    """Keras 2.13 EarlyStopping.on_epoch_end, including wait-counter order and the epoch>0 rule."""

    def __init__(self, monitor='val_loss', min_delta=0, patience=0, verbose=0, mode='auto',
                 baseline=None, restore_best_weights=False, start_from_epoch=0):
        super().__init__()
        self.monitor, self.patience, self.verbose = monitor, patience, verbose
        self.baseline, self.restore_best_weights = baseline, restore_best_weights
        self.start_from_epoch = start_from_epoch
        self.min_delta = abs(min_delta)
        if mode == 'max' or (mode == 'auto' and monitor.endswith('acc')):
            self.monitor_op = np.greater
        else:
            self.monitor_op = np.less
            self.min_delta *= -1
        self.wait = 0
        self.stopped_epoch = 0
        self.best = np.inf if self.monitor_op == np.less else -np.inf
        self.best_weights = None
        self.best_epoch = 0

    def on_train_begin(self, logs=None):
        self.wait = 0
        self.stopped_epoch = 0
        self.best = np.inf if self.monitor_op == np.less else -np.inf
        self.best_weights = None
        self.best_epoch = 0

    def _is_improvement(self, cur, ref):
        return self.monitor_op(cur - self.min_delta, ref)

    def on_epoch_end(self, epoch, logs=None):
        cur = (logs or {}).get(self.monitor)
        if cur is None or epoch < self.start_from_epoch:
            return
        if self.restore_best_weights and self.best_weights is None:
            self.best_weights = self.model.get_weights()
        self.wait += 1
        if self._is_improvement(cur, self.best):
            self.best = cur
            self.best_epoch = epoch
            if self.restore_best_weights:
                self.best_weights = self.model.get_weights()
            if self.baseline is None or self._is_improvement(cur, self.baseline):
                self.wait = 0
            return
        if self.wait >= self.patience and epoch > 0:
            self.stopped_epoch = epoch
            self.model.stop_training = True
            if self.restore_best_weights and self.best_weights is not None:
                if self.verbose:
                    print('Restoring model weights from the end of the best epoch: %d.'
                          % (self.best_epoch + 1))
                self.model.set_weights(self.best_weights)

    def on_train_end(self, logs=None):
        if self.stopped_epoch > 0 and self.verbose:
            print('Epoch %05d: early stopping' % (self.stopped_epoch + 1))
