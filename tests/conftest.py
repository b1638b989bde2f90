import glob
import os
import random
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the repo root and every examples/<family> directory (examples are imported by module name)
for p in [ROOT] + sorted(d for d in glob.glob(os.path.join(ROOT, "examples", "*")) if os.path.isdir(d)):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(autouse=True)
def _seed():
    random.seed(0)
    try:
        import numpy as np
        np.random.seed(0)
    except ImportError:
        pass
    try:
        import torch
        torch.manual_seed(0)
    except ImportError:
        pass
    yield
