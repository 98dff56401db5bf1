#!/bin/bash
# Session script (round 5): grid form (G workgroups per problem) of the small-batch OCP IPM: OCP GPU tests, probes with
# the grid on / off, stamps (workgroup 0 of problem 0).
O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 250 python -u lab/ric_pathcheck.py > $O/ric.log 2>&1 || { cat $O/ric.log; exit 7; }; cat $O/ric.log
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ocp_ipm.py tests/test_ocp_eq.py -m gpu > $O/pytest.log 2>&1; rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
export OCP_REPS=20
for gr in 0 1 16; do
  OCP_GRID=$gr timeout -k 10 200 python -u tools/ocp_probe.py 1 8 32 > $O/probe_g$gr.log 2>&1 || { cat $O/probe_g$gr.log; exit 9; }
  sed "s/^/G=$gr /" $O/probe_g$gr.log
done
CMPC_LIB=lab/_stamps/libcmpc_ocpstamps.so timeout -k 10 200 python -u tools/ocp_probe.py --stamps > $O/stamps.log 2>&1 || { cat $O/stamps.log; exit 8; }; cat $O/stamps.log
timeout -k 10 200 tests/cpp/bin/test_hpipm_interface > $O/cpp_mirror.log 2>&1; rc=$?; cat $O/cpp_mirror.log; exit $rc
