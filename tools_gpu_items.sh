#!/bin/bash
# GPU-box script: GPU tests, then the headline bench with the work-item fused kernel (default) and without
# (CMPC_ITEMS=0: k_solve64), alternating; a failing step ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; echo tests_rc=$rc; fatal $rc tests; [ $rc -ne 0 ] && exit 1
fi
for I in 1 0 1 0; do
  CMPC_ITEMS=$I timeout -k 10 200 python bench.py --cpu-sample 0 ${BENCH_ARGS:-} > $O/bench_i$I.json 2> $O/bench_i$I.err; rc=$?; fatal $rc bench; [ $rc -ne 0 ] && { tail -3 $O/bench_i$I.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_i$I.json'));print('items=$I',round(d['value']),{k:round(v,4) for k,v in d['stages_ms'].items()},round(d['ms_per_step'],4))"
done
