#!/bin/bash
# Session script (round 5): latency form of the OCP factorisation (ocp_chain.hpp): OCP GPU tests, B = 1 probe both
# paths, phase stamps.
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ocp_ipm.py tests/test_ocp_eq.py -m gpu > $O/pytest.log 2>&1; rc=$?; tail -6 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
export OCP_REPS=20
for c in 1 0; do
  OCP_CHAIN=$c timeout -k 10 200 python -u tools/ocp_probe.py 1 8 64 256 > $O/probe$c.log 2>&1 || { cat $O/probe$c.log; exit 9; }
  sed "s/^/chain$c /" $O/probe$c.log
done
CMPC_LIB=lab/_stamps/libcmpc_ocpstamps.so timeout -k 10 200 python -u tools/ocp_probe.py --stamps > $O/stamps.log 2>&1; cat $O/stamps.log
