#!/bin/bash
O=gpurun_out/r04ah; mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_ocp_ipm.py tests/test_ocp_eq.py -m gpu > $O/pytest.log 2>&1; rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 tests/cpp/bin/test_hpipm_interface > $O/cpp.log 2>&1; rc=$?; echo "cpp rc $rc"; tail -3 $O/cpp.log; [ $rc -eq 0 ] || exit $rc
export OCP_REPS=20
for i in 1 2; do
  for L in new:cheeta-mpc_amd/lib/libcmpc.so prev:lab/_ab/libcmpc_prev.so; do
    n=${L%%:*}; CMPC_LIB=${L#*:} timeout -k 10 200 python -u tools/ocp_probe.py 1 1024 > $O/$n$i.log 2>&1 || { cat $O/$n$i.log; exit 9; }
    sed "s/^/$n$i /" $O/$n$i.log
  done
done
