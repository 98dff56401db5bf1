#!/bin/bash
# Session script (round 5): the symmetric-sweep chain: OCP GPU tests, chain-only timing, B = 1 probe, stamps.
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ocp_ipm.py tests/test_ocp_eq.py -m gpu > $O/pytest.log 2>&1; rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
CMPC_LIB=lab/_stamps/libcmpc_ocpchain.so timeout -k 10 200 python -u tools/ocp_probe.py --chain > $O/chain.log 2>&1; cat $O/chain.log
export OCP_REPS=20
OCP_CHAIN=1 timeout -k 10 200 python -u tools/ocp_probe.py 1 64 256 > $O/probe1.log 2>&1 || { cat $O/probe1.log; exit 9; }
cat $O/probe1.log
CMPC_LIB=lab/_stamps/libcmpc_ocpstamps.so timeout -k 10 200 python -u tools/ocp_probe.py --stamps > $O/stamps.log 2>&1; cat $O/stamps.log
