"""Keras legacy optimizers (keras.optimizers.SGD / Adam / Adamax as constructed at
Model-96/train_96.py:99-103 and Model-88/train_88.py:323).  Descriptors only: the update runs in
libhpe.so's fused optimizer kernel (hpe_optim_step)."""


class Optimizer:
    kind = None

    def __init__(self, learning_rate=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-7, name=None, **kw):
        if learning_rate is None or float(learning_rate) < 0:
            raise ValueError('learning_rate must be >= 0, got %r' % (learning_rate,))
        self.learning_rate = float(learning_rate)
        self.beta_1, self.beta_2, self.epsilon = float(beta_1), float(beta_2), float(epsilon)
        self.name = name or type(self).__name__
        self.iterations = 0

    def get_config(self):
        return {'name': self.name, 'learning_rate': self.learning_rate, 'beta_1': self.beta_1,
                'beta_2': self.beta_2, 'epsilon': self.epsilon}


class SGD(Optimizer):
    kind = 'sgd'

    def __init__(self, learning_rate=0.01, momentum=0.0, nesterov=False, **kw):
        if momentum:
            raise ValueError('SGD momentum is not used by the reference (train_88.py:323)')
        super().__init__(learning_rate=learning_rate, **kw)


class Adam(Optimizer):
    kind = 'adam'


class Adamax(Optimizer):
    kind = 'adamax'


def get(identifier):
    if isinstance(identifier, Optimizer):
        return identifier
    if isinstance(identifier, str):
        m = {'sgd': SGD, 'adam': Adam, 'adamax': Adamax}
        if identifier.lower() in m:
            return m[identifier.lower()]()
    raise ValueError('Could not interpret optimizer identifier: %r' % (identifier,))
