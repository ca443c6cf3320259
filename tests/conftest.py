import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running")


def _have_gpu() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    # GPU tests fail loudly on a GPU box; on a CPU-only box they are skipped
    # only when explicitly deselected (-m "not gpu"), never silently passed.
    pass


@pytest.fixture(scope="session")
def repo_root():
    return ROOT


@pytest.fixture(scope="session")
def native():
    from bidirectional_bfs_amd import native as n

    return n


@pytest.fixture(scope="session")
def gpu_engine():
    import torch  # noqa: F401  (binds the HIP runtime first, like bench.py)

    from bidirectional_bfs_amd.ops import HipEngine

    return HipEngine(0)
