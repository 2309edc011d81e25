import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "ilqr.jl_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def pytest_collection_modifyitems(config, items):
    # GPU tests must not run (and must not be silently skipped into a pass) on CPU
    # unless explicitly selected: `-m gpu` on a box, `-m "not gpu"` here.
    pass


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no GPU is visible (run with -m 'not gpu' on CPU)")
    return torch.device("cuda", 0)
