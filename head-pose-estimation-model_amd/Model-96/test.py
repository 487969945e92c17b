"""evaluate_head_pose_model of Model-96/test.py:9-69 on the hpe runtime: load a model (converted
fixture / model saved by hpe / Keras .h5 via hpe.h5io), reshape the dataset's (N, 96) features to
(N, 1, 1, 96), predict on the GPU, per-angle MAE / MSE in yaw, pitch, roll order and their means,
printed to 4 decimals.  The wandb back-fill helper (:71-122) is out of scope (remote service)."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from hpe.data import evaluate_metrics  # noqa: E402
from hpe.model import load_model  # noqa: E402


def evaluate_head_pose_model(model_path, dataset_path):
    model = load_model(model_path)
    data = np.load(dataset_path)
    features, ground_truth = data['features'], data['poses']
    n, c = features.shape[0], features.shape[-1]
    predictions = model.predict(features.reshape(n, 1, 1, c), verbose=0)
    if predictions.shape != ground_truth.shape:
        predictions = predictions.reshape(n, 3)
    metrics = evaluate_metrics(predictions, ground_truth)
    print('Evaluation Results:')
    print('------------------')
    for title, key in (('Mean Absolute Error (MAE):', 'MAE'), ('\nMean Squared Error (MSE):', 'MSE')):
        print(title)
        for angle in ('yaw', 'pitch', 'roll'):
            print(f'  {angle}: {metrics[key][angle]:.4f}')
        print(f"  Average: {metrics[key]['average']:.4f}")
    return metrics


if __name__ == '__main__':
    if len(sys.argv) == 3:
        evaluate_head_pose_model(sys.argv[1], sys.argv[2])
