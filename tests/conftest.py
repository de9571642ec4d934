import json
import os
import sys
from functools import lru_cache

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, 'splendor-rl-gym_amd'), os.path.join(REPO, 'oracle')):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, 'tests', 'golden')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (run on the GPU box with -m gpu)')
    config.addinivalue_line('markers', 'slow: long-running parity case')


@lru_cache(maxsize=None)
def golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def golden_exists(name):
    return os.path.exists(os.path.join(GOLDEN, name))


@pytest.fixture(scope='session')
def tables():
    return golden('tables.json')
