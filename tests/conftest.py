import os
import random
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "examples", "gemm"), os.path.join(ROOT, "examples", "flash_attention")):
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
for _p in ("gemm_fp8", "deepseek_mla"):
    _d = os.path.join(ROOT, "examples", _p)
    if _d not in sys.path:
        sys.path.insert(0, _d)
