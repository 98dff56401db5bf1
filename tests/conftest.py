import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "cheeta-mpc_amd", "python"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device; runs through the C ABI")


# Under -x a failure hides every later test, so each BASELINE config's oracle-parity test runs first: config 1
# (CentoidMPCTest plumbing through the C++ mirror), configs 2 / 3 / 5 and config 4's per-GPU share at full size,
# config 4 whole on one GPU and sharded over two ranks, the goldens; then the rows new since the last driver run
# (UpdateMPC foot semantics, the equality-constrained HpipmInterface path, the SQP); then the rest in file order.
_FIRST = ("test_gpu_parity.py::test_cpp_centroidal_mpc_driver", "test_full_size.py::test_full_size_config",
          "test_multi_rank_gpu.py::test_config4_full_batch_one_gpu",
          "test_multi_rank_gpu.py::test_two_rank_hip_shards_gather_bit_exact",
          "test_gpu_parity.py::test_device_matches_golden_fp64", "test_gpu_parity.py::test_device_foot_semantics",
          "test_ocp_eq.py::", "test_hpipm_eq_riccati.py::", "test_sqp.py::", "test_feet.py::")


def pytest_collection_modifyitems(session, config, items):
    def rank(item):
        nid = item.nodeid.split("/")[-1]
        for k, p in enumerate(_FIRST):
            if nid.startswith(p):
                return k
        return len(_FIRST)
    items[:] = sorted(items, key=rank)  # stable: file order inside each group


def pytest_terminal_summary(terminalreporter):
    """Name the build the session ran (source hash of libcmpc.so and its md5) at the end of every log."""
    try:
        import hashlib
        import cheeta_mpc
        with open(cheeta_mpc.LIB_PATH, "rb") as f:
            md5 = hashlib.md5(f.read()).hexdigest()
        terminalreporter.write_line(f"cmpc build: {cheeta_mpc.lib().cmpc_version().decode()}, libcmpc.so md5 {md5}")
    except Exception as e:  # noqa: BLE001 - informational only
        terminalreporter.write_line(f"cmpc build: unavailable ({e!r})")


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
