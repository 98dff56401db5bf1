import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "cheeta-mpc_amd", "python"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device; runs through the C ABI")


@pytest.fixture(scope="session")
def cm():
    import cheeta_mpc
    if cheeta_mpc.device_count() == 0:
        pytest.fail("gpu test scheduled but no HIP device is visible")
    return cheeta_mpc


@pytest.fixture(scope="session")
def op():
    import oracle_py
    return oracle_py


@pytest.fixture(scope="session")
def cmh():
    """The package for host-only calls (no device needed: defaults, built-in tables, struct layouts)."""
    import cheeta_mpc
    return cheeta_mpc
