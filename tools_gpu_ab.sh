#!/bin/bash
# GPU-box script: GPU tests, then the headline bench with the fused n <= 64 kernel (default) and without
# (CMPC_FUSED=0), then rocprofv3 kernel stats of the fused bench. A failing step ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -4 $O/gpu_tests.log; echo tests_rc=$rc; fatal $rc tests; [ $rc -ne 0 ] && exit 1
fi
for F in 1 0 1 0; do
  CMPC_FUSED=$F timeout -k 10 200 python bench.py --cpu-sample 0 ${BENCH_ARGS:-} > $O/bench_f$F.json 2> $O/bench_f$F.err; rc=$?; fatal $rc bench; [ $rc -ne 0 ] && { tail -3 $O/bench_f$F.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_f$F.json'));print('fused=$F',round(d['value']),{k:round(v,4) for k,v in d['stages_ms'].items()},round(d['ms_per_step'],4))"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_ab -o run --output-format csv -- python3 $R/bench.py --steps 10 --cpu-sample 0 ${BENCH_ARGS:-} > $O/prof_ab.log 2>&1 || exit 1
cut -d, -f1-4 $O/prof_ab/run_kernel_stats.csv | head -8
