import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "slow: long-running")


def gpu_available() -> bool:
    try:
        import torch  # noqa: F401  (device probe only; the engine itself is torch-free)

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def built():
    """Build the product library and the oracle once per session (no-op when up to date)."""
    import subprocess

    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "matching_engine_amd")], check=True)
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "lib"], check=True, stdout=subprocess.DEVNULL)
    return True
