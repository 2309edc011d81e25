import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "ilqr.jl_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


# GPU modules in the order they run: the BASELINE configs and the headline first, so
# that `-m gpu -x` stopping on a family's unit test cannot hide them; then the LQ
# parity suite, the 2-link family, tiles, layouts, and the chain family last.
_ORDER = ("test_gpu_configs", "test_gpu_headline", "test_gpu_line_search", "test_gpu_history", "test_gpu_multi", "test_gpu_parity", "test_gpu_twolink",
          "test_gpu_tiles", "test_gpu_julia_layout", "test_gpu_julia_resident", "test_gpu_helpers",
          "test_gpu_cost_functions", "test_gpu_chain")


def pytest_collection_modifyitems(config, items):
    # GPU tests must not run (and must not be silently skipped into a pass) on CPU
    # unless explicitly selected: `-m gpu` on a box, `-m "not gpu"` here.
    def key(item):
        mod = item.module.__name__.rsplit(".", 1)[-1] if item.module else ""
        return _ORDER.index(mod) if mod in _ORDER else len(_ORDER)
    items.sort(key=key)  # stable: file order within a module is kept


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no GPU is visible (run with -m 'not gpu' on CPU)")
    return torch.device("cuda", 0)
