import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, 'tests', 'golden')
for p in (ROOT, GOLDEN):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a visible MI355X (HIP device)')
    config.addinivalue_line('markers', 'slow: large synthetic sizes')


@pytest.fixture(scope='session')
def golden_dir():
    return GOLDEN
