#!/bin/bash
# GPU-box script (round 5): rocprofv3 kernel stats of configs 3 and 5 (bench.py lines of profiles/r05_c3.json /
# r05_c5.json), to split each step by kernel.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/c35_r05; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python3 $R/bench.py --horizon 20 --precision f32 --steps 50 --warmup 10 --cpu-sample 0 > $O/c3.log 2>&1 || { tail -5 $O/c3.log; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o run --output-format csv -- python3 $R/bench.py --gait 1 --steps 50 --warmup 10 --cpu-sample 0 > $O/c5.log 2>&1 || { tail -5 $O/c5.log; exit 1; }
tail -1 $O/c3.log; tail -1 $O/c5.log; find $O -name "*kernel_stats.csv"
