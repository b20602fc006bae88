import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def pytest_make_parametrize_id(config, val, argname):
    """Readable ids for torch dtypes (``float16`` instead of ``dtype2``), so ``-k float16``
    selects the fp16 cases."""
    import torch
    if isinstance(val, torch.dtype):
        return str(val).replace("torch.", "")
    return None
