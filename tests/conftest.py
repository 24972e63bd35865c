import os
import sys

import pytest

# the tests switch kernel forms and gates through their PPOX_* variables (native.ab_env, common.h ppox::ab_env):
# read only under PPOX_AB=1 (before the package is imported; inherited by the tests' rank processes)
os.environ.setdefault("PPOX_AB", "1")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ppo-exploration_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture
def golden():
    import numpy as np

    def load(name):
        return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    return load
