#!/bin/bash
# GPU-box script: GPU tests, then the batched SQP bench line (N = 10 trot and mixed gait). A failing step ends it.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; fatal $rc tests; [ $rc -ne 0 ] && { grep -E 'FAIL|Error|assert' $O/gpu_tests.log | head -20; exit 1; }
for g in 0 1; do
  timeout -k 10 200 python bench.py --cpu-sample 0 --sqp-iters 10 --gait $g --steps 10 > $O/sqp_g$g.json 2> $O/sqp_g$g.err; rc=$?
  fatal $rc sqp$g; [ $rc -ne 0 ] && { tail -3 $O/sqp_g$g.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/sqp_g$g.json'));print($g, round(d['value']), d.get('solver'))"
done
