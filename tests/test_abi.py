"""CPU suite: the C-ABI library (cheeta-mpc_amd/lib/libcmpc.so) loads, exports every symbol include/*.h declares,
and its host-side defaults/struct layouts match the reference (no compute call needs a GPU here)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions(header):
    txt = open(header).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\**\s*(cmpc_[a-z_0-9]+)\s*\(", txt, flags=re.M)
    return sorted(set(names))


def test_library_exports_every_declared_symbol():
    import cheeta_mpc
    L = cheeta_mpc.lib()
    names = declared_functions(os.path.join(ROOT, "include", "cmpc", "cmpc.h"))
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    out = subprocess.check_output(["nm", "-D", "--defined-only", cheeta_mpc.LIB_PATH], text=True)
    for n in names:
        assert re.search(rf"\bT {n}$", out, flags=re.M), n


def test_settings_defaults_match_hpipm_interface():
    import cheeta_mpc
    s = cheeta_mpc.default_settings()
    # hpipm_interface::Settings (HpipmInterfaceSettings.h:44-57)
    assert (s.iter_max, s.alpha_min, s.mu0, s.tol_stat, s.tol_eq, s.tol_ineq, s.tol_comp, s.reg_prim) == \
        (30, 1e-12, 10.0, 1e-6, 1e-8, 1e-8, 1e-8, 1e-12)
    assert (s.warm_start, s.pred_corr, s.ric_alg) == (0, 1, 0)
    assert s.hpipm_mode == 1  # hpipm_mode::SPEED, same numbering as the mirrored enum (HpipmInterface.h)


@pytest.mark.parametrize("field,value", [("pred_corr", 0), ("hpipm_mode", 4), ("hpipm_mode", -1), ("ric_alg", 2),
                                         ("warm_start", 2), ("tol_stat", 0.0), ("mu0", -1.0), ("iter_max", -1)])
def test_unsupported_settings_rejected(field, value):
    """Settings the build does not implement are refused (CMPC_ERR_ARG) before any device call, not ignored."""
    import ctypes as C
    import cheeta_mpc
    s = cheeta_mpc.default_settings(**{field: value})
    m = cheeta_mpc.default_model(10)
    ctx = C.c_void_p()
    assert cheeta_mpc.lib().cmpc_create(C.byref(m), C.byref(s), 0, 16, None, C.byref(ctx)) == -1
    assert cheeta_mpc.lib().cmpc_set_settings(None, C.byref(s)) == -1


def test_model_default_is_centoid_mpc_test(op):
    import cheeta_mpc
    m = cheeta_mpc.default_model(6)
    o = op.default_model(6)
    assert m.N == 6 and m.n_legs == 4 and m.mass == 8.0 and m.dt == 0.01
    assert list(m.weights) == list(o.weights)
    assert list(m.mu) == [0.8] * 4
    assert list(m.force_ub) == [5000.0] * 4 + [8.0 * 9.81 * 4]


def test_struct_layouts_match_c(tmp_path):
    import cheeta_mpc
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "cmpc/cmpc.h"\nint main(void){printf("%zu %zu %zu %zu\\n",'
                   ' sizeof(cmpc_model), sizeof(cmpc_settings), offsetof(cmpc_model, weights),'
                   ' offsetof(cmpc_settings, warm_start)); return 0;}\n')
    exe = tmp_path / "sz"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    a, b, c, d = (int(v) for v in subprocess.check_output([str(exe)], text=True).split())
    assert a == C.sizeof(cheeta_mpc.Model) and b == C.sizeof(cheeta_mpc.Settings)
    assert c == cheeta_mpc.Model.weights.offset and d == cheeta_mpc.Settings.warm_start.offset


def test_memsize_and_arg_checks():
    import cheeta_mpc
    L = cheeta_mpc.lib()
    m = cheeta_mpc.default_model(10)
    s64 = L.cmpc_memsize(C.byref(m), 0, 4096)
    s32 = L.cmpc_memsize(C.byref(m), 1, 4096)
    assert s64 > 4096 * 128 * 128 * 8 and s32 < s64
    bad = cheeta_mpc.default_model(10)
    bad.n_legs = 2
    assert L.cmpc_memsize(C.byref(bad), 0, 16) == 0
    ctx = C.c_void_p()
    assert L.cmpc_create(C.byref(bad), None, 0, 16, None, C.byref(ctx)) == -1  # CMPC_ERR_ARG
    assert L.cmpc_ocp_solve_batch_host(1, 0, 3, None, None, None, None, None, None) == -1
    assert L.cmpc_status_string(5) == b"INVALID_CONTACT" and L.cmpc_status_string(0) == b"SUCCESS"
    nu = np.array([2, 0, 2], dtype=np.int32)
    assert L.cmpc_ocp_record_size(3, 3, nu.ctypes.data_as(C.c_void_p)) == \
        cheeta_mpc.lib().cmpc_ocp_record_size(3, 3, nu.ctypes.data_as(C.c_void_p))


def test_ocp_record_size_matches_oracle(op):
    import cheeta_mpc
    nu = np.array([2, 0, 2, 1], dtype=np.int32)
    a = cheeta_mpc.lib().cmpc_ocp_record_size(4, 3, nu.ctypes.data_as(C.c_void_p))
    b = op.lib().oracle_ocp_record_size(4, 3, nu.ctypes.data_as(C.POINTER(C.c_int)))
    assert a == b


def test_no_device_is_reported_not_faked():
    import cheeta_mpc
    if cheeta_mpc.device_count() > 0:
        pytest.skip("a GPU is visible")
    m = cheeta_mpc.default_model(10)
    ctx = C.c_void_p()
    assert cheeta_mpc.lib().cmpc_create(C.byref(m), None, 0, 16, None, C.byref(ctx)) == -4  # CMPC_ERR_NO_DEVICE


def test_cpp_mirror_headers_compile(tmp_path):
    src = tmp_path / "t.cpp"
    src.write_text('#include "cheeta_mpc/CentroidalMPC.h"\n#include "hpipm_catkin/HpipmInterface.h"\n'
                   'int main(){ ocs2::HpipmInterface::OcpSize s(5,3,2); return s.numInputs.back(); }\n')
    subprocess.check_call(["g++", "-std=c++17", "-fsyntax-only", "-I", os.path.join(ROOT, "include"), str(src)])


def test_step_ratio_extreme_fp32_values():
    """The IPM kernels' fraction-to-boundary selection (csrc/step_ratio.hpp) compared in double: fp32 slacks and
    directions near 1e-20 / 1e+20 still select the binding candidate (host build of the same header)."""
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp"), "bin/test_step_ratio"])
    out = subprocess.check_output([os.path.join(ROOT, "tests", "cpp", "bin", "test_step_ratio")], text=True)
    assert "step_ratio: ok" in out, out


def test_riccati_getter_clamp_near_singular_R():
    """The HpipmInterface mirror's optional Lr clamp (setRiccatiMinimumEigenvalue; the reference's
    LinearAlgebra::setTriangularMinimumEigenvalues in every getter, HpipmInterface.cpp:340, :357, :379, :419) on a stage
    with a near-singular R + B'PB (Lr(0,0) = 1e-7): the clamp rule, and K re-derived as -Lc^-T Ls' (:361) matching an
    independent solve and the closed form of the clamped row (host build of the header, no device)."""
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp"), "bin/test_riccati_clamp"])
    out = subprocess.check_output([os.path.join(ROOT, "tests", "cpp", "bin", "test_riccati_clamp")], text=True)
    assert "riccati_clamp: ok" in out, out


def test_path_option_constants_match_header():
    """cheeta_mpc.PATH_* mirror enum cmpc_path_option of include/cmpc/cmpc.h (cmpc_set_path / cmpc_get_path)."""
    import cheeta_mpc
    txt = open(os.path.join(ROOT, "include", "cmpc", "cmpc.h")).read()
    body = re.search(r"enum cmpc_path_option\s*\{(.*?)\}", txt, flags=re.S).group(1)
    enum = {k: int(v) for k, v in re.findall(r"CMPC_PATH_([A-Z0-9]+)\s*=\s*(\d+)", body)}
    assert set(enum) == {"FUSED64", "FUSED128", "DIRECT", "RICCATI", "IPM72"}
    for k, v in enum.items():
        assert getattr(cheeta_mpc, "PATH_" + k) == v, k


def test_status_strings_cover_every_code(cmh):
    """cmpc_status_string names every cmpc_qp_status (INFEASIBLE_STEP printed as UNKNOWN) and the Python
    table agrees."""
    L = cmh.lib()
    for code, name in cmh.STATUS.items():
        assert L.cmpc_status_string(code).decode() == name
    assert L.cmpc_status_string(7).decode() == "INFEASIBLE_STEP"


@pytest.mark.gpu
def test_fused64_off_refused_while_riccati_path_is_on(cm):
    """CMPC_PATH_RICCATI = 1 runs on the fused path, so switching FUSED64 off under it is refused instead of
    silently skipping the stage-wise kernel."""
    eng = cm.Engine(cm.default_model(10), max_batch=8)
    eng.set_path(cm.PATH_RICCATI, 1)
    with pytest.raises(RuntimeError):
        eng.set_path(cm.PATH_FUSED64, 0)
    assert eng.get_path(cm.PATH_FUSED64) == 1 and eng.get_path(cm.PATH_RICCATI) == 1
    eng.set_path(cm.PATH_RICCATI, 0)
    eng.set_path(cm.PATH_FUSED64, 0)
    assert eng.get_path(cm.PATH_FUSED64) == 0
