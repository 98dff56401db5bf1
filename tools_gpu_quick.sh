#!/bin/bash
# GPU-box script: GPU parity tests, then the bench sweep (tools_bench_sweep.sh). Stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -15 gpurun_out/gpu_tests.log; echo tests_rc=$rc
[ $rc -ne 0 ] && exit 1
bash tools_bench_sweep.sh
