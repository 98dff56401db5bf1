#!/bin/bash
# GPU-box script: GPU tests, then config 3 (N = 20 fp32) with the 128 class on four (fused / two launches) and two
# waves per QP, alternating; then configs 2 and 5 as regression checks. A failing step ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; fatal $rc tests; [ $rc -ne 0 ] && { grep -E 'FAIL|Error|assert' $O/gpu_tests.log | head -20; exit 1; }
AB="w4fused=CMPC_W128=4;w4two=CMPC_FUSED128=0;w2=CMPC_W128=2" ROUNDS=2 BENCH_ARGS="--horizon 20 --precision f32 --steps 20" bash tools_gpu_abenv.sh || exit 1
AB="head=CMPC_W128=4" ROUNDS=1 BENCH_ARGS="--steps 30" bash tools_gpu_abenv.sh || exit 1
AB="c5=CMPC_W128=4" ROUNDS=1 BENCH_ARGS="--gait 1 --steps 20" bash tools_gpu_abenv.sh || exit 1
