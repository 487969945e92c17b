"""Model-96/utilities.py of the reference on the hpe runtime: the drivers' ``from utilities import ...``
resolves here; the implementation is shared with the other model family in hpe/utilities.py."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hpe.utilities import (WandbCallback, analyze_angle_distributions, load_dataset,  # noqa: E402,F401
                           load_dataset_with_weights, load_model_from_json)
