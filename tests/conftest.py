import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(autouse=True)
def _fresh_dropout_salts():
    """Every test builds its models from the first dropout salt (sparkmi/ops/rng.py: salts are a
    process-global counter), so a test's dropout masks — its problem instance — do not depend on
    how many models earlier tests built (a trajectory test with a loss spike passed alone and
    failed after the rest of its file)."""
    from sparkmi.ops import rng
    rng.reset_salts()
    yield
