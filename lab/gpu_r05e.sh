#!/bin/bash
# Session script (round 5): chain prefetch without early waits — chain-only timing (normal / no-fetch ceiling),
# stamps of the grid form, probes.
O=gpurun_out/r05e; mkdir -p $O
CMPC_LIB=lab/_stamps/libcmpc_ocpchain.so timeout -k 10 200 python -u tools/ocp_probe.py --chain > $O/chain.log 2>&1 || { cat $O/chain.log; exit 6; }; cat $O/chain.log
CMPC_LIB=lab/_stamps/libcmpc_ocpnofetch.so timeout -k 10 200 python -u tools/ocp_probe.py --chain > $O/nofetch.log 2>&1 || { cat $O/nofetch.log; exit 5; }; sed 's/^/nofetch /' $O/nofetch.log
OCP_REPS=20 timeout -k 10 200 python -u tools/ocp_probe.py 1 8 32 > $O/probe.log 2>&1 || { cat $O/probe.log; exit 9; }; cat $O/probe.log
CMPC_LIB=lab/_stamps/libcmpc_ocpstamps.so timeout -k 10 200 python -u tools/ocp_probe.py --stamps > $O/stamps.log 2>&1 || { cat $O/stamps.log; exit 8; }; cat $O/stamps.log
