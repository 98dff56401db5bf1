#!/bin/bash
# GPU-box script: GPU tests, then three headline bench lines and one line each for configs 3 and 5, N = 20 fp64 and
# N = 10 all-stance fp64. A failing step ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -2 gpurun_out/gpu_tests.log; fatal $rc tests; [ $rc -ne 0 ] && { grep -E 'FAIL|Error|assert' gpurun_out/gpu_tests.log | head; exit 1; }
for cfg in "" "" "" "--gait 1" "--horizon 20 --precision f32" "--horizon 20" "--all-stance"; do
  timeout -k 10 120 python bench.py --cpu-sample 0 --steps 30 $cfg > gpurun_out/b.json 2>gpurun_out/b.err; rc=$?; fatal $rc "bench $cfg"; [ $rc -ne 0 ] && { tail -3 gpurun_out/b.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/b.json')); print('[$cfg]', round(d['value']), {k: round(v,4) for k,v in d['stages_ms'].items()}, d['solver']['mean_iters'])"
done
