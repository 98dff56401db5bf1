#!/bin/bash
# GPU-box script: headline bench (no CPU baseline) + rocprofv3 kernel stats of the same command.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 200 python bench.py --cpu-sample 0 ${BENCH_ARGS:-} > $O/bench_q.json 2> $O/bench_q.err; rc=$?; echo bench_rc=$rc
python3 -c "import json;d=json.load(open('$O/bench_q.json'));print(d['value'],d['stages_ms'],d['roofline']['frac'])"
[ $rc -ne 0 ] && exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_q -o run --output-format csv -- python3 $R/bench.py --steps 10 --cpu-sample 0 ${BENCH_ARGS:-} > $O/prof_q.log 2>&1 || exit 1
cut -d, -f1-4 $O/prof_q/run_kernel_stats.csv | head -8
