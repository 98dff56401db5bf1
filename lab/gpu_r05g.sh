#!/bin/bash
# Session script (round 5): stamps of the grid-form chain (wave 0 phases, wave 1 load span), chain-only timing
O=gpurun_out/r05g; mkdir -p $O
CMPC_LIB=lab/_stamps/libcmpc_ocpstamps.so timeout -k 10 200 python -u tools/ocp_probe.py --stamps > $O/stamps.log 2>&1 || { cat $O/stamps.log; exit 8; }; cat $O/stamps.log
CMPC_LIB=lab/_stamps/libcmpc_ocpchain.so timeout -k 10 200 python -u tools/ocp_probe.py --chain > $O/chain.log 2>&1 || { cat $O/chain.log; exit 6; }; cat $O/chain.log
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ocp_ipm.py tests/test_ocp_eq.py -m gpu > $O/pytest.log 2>&1; rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
OCP_REPS=20 timeout -k 10 200 python -u tools/ocp_probe.py 1 8 32 > $O/probe.log 2>&1 || { cat $O/probe.log; exit 9; }; cat $O/probe.log
