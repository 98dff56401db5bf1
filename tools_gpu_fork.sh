#!/bin/bash
# GPU-box script: forked bigger classes (CMPC_FORK=1) parity, the full GPU suite, then A/B on the headline, config 5,
# config 3 and N = 20 fp64, alternating. A failing step ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 150 python -u -m pytest tests/test_fused128.py -m gpu -x -v --timeout 60 --timeout-method thread > $O/gpu_tests_fork.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error" $O/gpu_tests_fork.log | tail -12; fatal $rc fork_tests; [ $rc -ne 0 ] && { tail -30 $O/gpu_tests_fork.log; exit 1; }
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -2 $O/gpu_tests.log; fatal $rc tests; [ $rc -ne 0 ] && { grep -E 'FAIL|Error|assert' $O/gpu_tests.log | head -20; exit 1; }
AB="hfork=CMPC_FORK=1;hbase=CMPC_FORK=0" ROUNDS=3 BENCH_ARGS="--steps 30" bash tools_gpu_abenv.sh || exit 1
AB="c5fork=CMPC_FORK=1;c5base=CMPC_FORK=0" ROUNDS=2 BENCH_ARGS="--gait 1 --steps 20" bash tools_gpu_abenv.sh || exit 1
AB="c3fork=CMPC_FORK=1;c3base=CMPC_FORK=0" ROUNDS=2 BENCH_ARGS="--horizon 20 --precision f32 --steps 20" bash tools_gpu_abenv.sh || exit 1
AB="n20fork=CMPC_FORK=1;n20base=CMPC_FORK=0" ROUNDS=1 BENCH_ARGS="--horizon 20 --steps 10" bash tools_gpu_abenv.sh || exit 1
