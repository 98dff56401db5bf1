#!/bin/bash
# GPU session script (round 4): OCP + full GPU tests, C++ mirror, Riccati probe, config 3 / 5 / headline benches with
# the 128-class LDS-layout change, MINB 4 vs 3 for the fused fp32 128 class.
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > $O/r04d_pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -8 $O/r04d_pytest.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 200 tests/cpp/bin/test_hpipm_interface > $O/r04d_cpp.log 2>&1
rc=$?; echo "cpp rc $rc"; tail -6 $O/r04d_cpp.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 120 python -u tools/ric_probe.py --gpu > $O/r04d_ric_probe.log 2>&1 && cat $O/r04d_ric_probe.log || exit 1
timeout -k 10 300 python -u bench.py --horizon 20 --precision f32 --steps 100 --warmup 20 --cpu-sample 0 > $O/r04d_c3.json 2> $O/r04d_c3.err && tail -1 $O/r04d_c3.json | cut -c1-400 || exit 1
CMPC_LIB=lab/_ab/libcmpc_minb3.so timeout -k 10 300 python -u bench.py --horizon 20 --precision f32 --steps 100 --warmup 20 --cpu-sample 0 > $O/r04d_c3_minb3.json 2> $O/r04d_c3_minb3.err && tail -1 $O/r04d_c3_minb3.json | cut -c1-400 || exit 1
timeout -k 10 300 python -u bench.py --gait 1 --steps 100 --warmup 20 --cpu-sample 0 > $O/r04d_c5.json 2> $O/r04d_c5.err && tail -1 $O/r04d_c5.json | cut -c1-400 || exit 1
timeout -k 10 300 python -u bench.py --steps 200 --warmup 50 --cpu-sample 0 > $O/r04d_c2.json 2> $O/r04d_c2.err && tail -1 $O/r04d_c2.json | cut -c1-400
