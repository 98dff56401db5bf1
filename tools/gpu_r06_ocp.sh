#!/bin/bash
# GPU-box script (round 6): the OCP GPU tests (test_ocp_*, the C++ HpipmInterface mirror) and the B = 1 OCP bench lines
# (projected / rows, with the C++ mirror tick). Every GPU step has its own time limit; a fault / abort / time-out ends
# the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/${OUT:-r06_ocp}; mkdir -p $O; cd $R
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
if [ -z "$NO_TESTS" ]; then
timeout -k 10 400 python -u -m pytest tests -m gpu -q -k "ocp or hpipm or riccati" --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; fatal $rc tests
fi
b() { local n=$1; shift; timeout -k 10 300 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err; local rc=$?; fatal $rc $n
      python3 -c "import json;d=json.loads(open('$O/$n.json').read().strip().split(chr(10))[-1]);t=d.get('tick') or {};print('$n',round(d['value']),d['unit'],round(d['ms_per_step'],4),d.get('ms_per_solve_b1'),t.get('tick_ms_median'),t.get('kernel_ms_median'),t.get('feedback_ms_median'))" || tail -3 $O/$n.err; }
b ocp_projected_b1 --ocp projected --batch 1 --steps 200 --warmup 20 --cpu-sample 0
b ocp_rows_b1 --ocp rows --batch 1 --steps 30 --warmup 3 --cpu-sample 0
echo all_done
