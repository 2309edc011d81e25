"""Every BASELINE.json configuration on the GPU against the oracle (tests/configs.py).
Collected before every other GPU module (tests/conftest.py), so `pytest -m gpu -x`
pins configs 1-5 even when a family's unit tests would stop the run later."""
import pytest

import configs

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("check", configs.ALL, ids=lambda f: f.__name__)
def test_baseline_config_vs_oracle(gpu, check):
    errs = check()
    print(" ".join(f"{k}={v:.2e}" for k, v in errs.items()))
