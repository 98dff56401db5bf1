"""Source compatibility of the C++ boundary with the reference's value types, checked by compilation on the CPU.

The reference's callers use Eigen (CentroidalMPC.h:26-32: Eigen::VectorXd) and ocs2_core (HpipmInterface.h:38:
<ocs2_core/Types.h>). This image has neither, so tests/cpp carries mocks with their API and storage rules (private
storage, no zero-initialising sizing constructors); the mirrors and the caller-style drivers must build against them
as well as against the stand-ins, with the same sources and only the include path changed. The GPU runs of the
resulting binaries are in test_gpu_parity.py."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(ROOT, "tests", "cpp")


def test_mirrors_compile_against_eigen_and_ocs2_shaped_types(tmp_path):
    out = str(tmp_path)
    r = subprocess.run(["make", "-s", "-C", CPP, f"OUT={out}", f"{out}/centroid_mpc_test_eigen",
                        f"{out}/test_hpipm_interface_ocs2", f"{out}/centroid_mpc_test", f"{out}/test_hpipm_interface"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    for b in ("centroid_mpc_test_eigen", "test_hpipm_interface_ocs2", "centroid_mpc_test", "test_hpipm_interface"):
        assert os.path.exists(os.path.join(out, b))


def test_host_mirrors_do_not_reach_into_storage():
    """The mirrors touch the value types only through rows() / cols() / size() / data() / resize() / operator():
    no stand-in-only members (the mock's storage is private, so the compile above enforces it; this keeps the
    sources honest for a reader too)."""
    for f in ("HpipmInterface.cpp", "CentroidalMPC.cpp"):
        src = open(os.path.join(ROOT, "cheeta-mpc_amd", "host", f)).read()
        for bad in (".a.", ".v.", ".a[", ".v[", ".a)", ".v)"):
            assert bad not in src, (f, bad)
