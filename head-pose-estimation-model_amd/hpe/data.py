"""Dataset helpers of the reference: utilities.load_dataset (Model-88/utilities.py:35-38,
Model-96/utilities.py:31-34) and sklearn's train_test_split(test_size=0.2, random_state=42)
(train_96.py:142-146), restated: perm = RandomState(seed).permutation(n), test = perm[:ceil(.2 n)]."""
import math

import numpy as np


def load_dataset(dataset_path):
    """Load the dataset containing features and poses."""
    data = np.load(dataset_path)
    return data['features'], data['poses']


def train_test_split(*arrays, test_size=0.2, random_state=None, shuffle=True):
    n = len(arrays[0])
    for a in arrays:
        if len(a) != n:
            raise ValueError('Found input variables with inconsistent numbers of samples')
    n_test = int(math.ceil(test_size * n)) if isinstance(test_size, float) else int(test_size)
    if shuffle:
        perm = np.random.RandomState(random_state).permutation(n)
    else:
        perm = np.arange(n)
    test, train = perm[:n_test], perm[n_test:]
    out = []
    for a in arrays:
        out += [a[train], a[test]]
    return out


def evaluate_metrics(predictions, ground_truth):
    """Metric block of evaluate_head_pose_model (Model-96/test.py:41-54)."""
    predictions = np.asarray(predictions).reshape(-1, 3)
    ground_truth = np.asarray(ground_truth).reshape(-1, 3)
    mae_pa = np.mean(np.abs(predictions - ground_truth), axis=0)
    mse_pa = np.mean(np.square(predictions - ground_truth), axis=0)
    names = ['yaw', 'pitch', 'roll']
    m = {'MAE': {names[i]: float(mae_pa[i]) for i in range(3)},
         'MSE': {names[i]: float(mse_pa[i]) for i in range(3)}}
    m['MAE']['average'] = float(np.mean(mae_pa))
    m['MSE']['average'] = float(np.mean(mse_pa))
    return m
