import os
import sys

import numpy as np
import pytest

# pytest-xdist: N workers x (all cores) OpenMP threads spin against each other and
# slow the CPU learner tests down ~100x; give each worker a fair share instead
if os.environ.get("PYTEST_XDIST_WORKER") and "OMP_NUM_THREADS" not in os.environ:
    _n = int(os.environ.get("PYTEST_XDIST_WORKER_COUNT", "1"))
    os.environ["OMP_NUM_THREADS"] = str(max(1, (os.cpu_count() or 1) // max(1, _n)))
    # estimators that pin num_threads (sklearn n_jobs=None -> physical cores) still
    # oversubscribe: idle OpenMP threads must sleep, not spin
    os.environ.setdefault("OMP_WAIT_POLICY", "PASSIVE")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X (gfx950) GPU and the HIP kernels")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def lgb():
    import lambdagap_amd

    return lambdagap_amd


@pytest.fixture(scope="session")
def gpu_required(lgb):
    """GPU tests fail loudly (never skip) when the device path is unavailable."""
    n = lgb.device_count()
    assert n >= 1, "GPU test requested but the native library sees no gfx950 device"
    return n


@pytest.fixture
def rng():
    return np.random.default_rng(12345)
