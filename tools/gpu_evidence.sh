#!/bin/bash
# GPU-box script: the evidence that does not depend on PMC passes (libcmpc.so unchanged since the stamped summaries):
# GPU tests, smoke, the headline bench with the CPU baseline, rocprofv3 kernel stats of the same bench command.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/evidence; mkdir -p $O; cd $R
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -2 $O/gpu_tests.log; fatal $rc tests; [ $rc -ne 0 ] && exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; fatal $rc smoke
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?; echo bench_rc=$rc; fatal $rc bench; [ $rc -ne 0 ] && exit 1
python3 -c "import json;d=json.load(open('$O/bench.json'));print(round(d['value']),d['stages_ms'],d['roofline']['frac'],d['cpu_baseline']['value'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --cpu-sample 0 > $O/prof.log 2>&1; rc=$?; fatal $rc prof; [ $rc -ne 0 ] && exit 1
echo all_done
