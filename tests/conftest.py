import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'head-pose-estimation-model_amd'), os.path.dirname(__file__)):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs the HIP path)')


@pytest.fixture(scope='session')
def golden_dir():
    return GOLDEN
