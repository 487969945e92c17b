"""hpe — MI355X-native head-pose regression hot path (Model-88 / Model-96 regressors of
Maaz77/Head-Pose-Estimation-Model): Keras-compatible host API over libhpe.so (HIP, gfx950)."""
from . import keras  # noqa: F401
from .data import load_dataset, train_test_split  # noqa: F401
from .model import Model, load_model, model_from_config  # noqa: F401
from .random import set_seed  # noqa: F401

__all__ = ['keras', 'Model', 'load_model', 'model_from_config', 'load_dataset',
           'train_test_split', 'set_seed']
