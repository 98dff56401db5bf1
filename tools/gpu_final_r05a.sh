#!/bin/bash
# GPU-box script (round 5 final evidence, part A): GPU tests, smoke, the headline bench with the CPU baseline and the
# 50 Hz cadence line, configs 3 / 5, the OCP bench lines (projected / rows at B = 1 with the C++ mirror tick and the
# single-thread CPU latency, and at B = 4096), rocprofv3 kernel stats of the headline and of the B = 1 OCP solves.
# ONLY_OCP=1: the OCP lines and profiles only. Every GPU step has its own time limit; a fault / abort / time-out ends
# the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/final_r05; mkdir -p $O; cd $R
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
if [ -z "$ONLY_OCP" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; fatal $rc tests
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; fatal $rc smoke
fi
b() { local n=$1; shift; timeout -k 10 300 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err; local rc=$?; fatal $rc $n
      python3 -c "import json;d=json.loads(open('$O/$n.json').read().strip().split(chr(10))[-1]);print('$n',round(d['value']),d['unit'],round(d['ms_per_step'],4),d.get('ms_per_solve_b1'),d.get('ms_per_solve_b1_host_path'),(d.get('tick') or {}).get('tick_ms_median'),d['roofline']['frac'] if d.get('roofline') else None)" || tail -3 $O/$n.err; }
if [ -z "$ONLY_OCP" ]; then
b bench --cadence 20
b c3 --horizon 20 --precision f32 --steps 100 --warmup 20 --cpu-sample 0
b c5 --gait 1 --steps 100 --warmup 20 --cpu-sample 0
fi
b ocp_projected_b1 --ocp projected --batch 1 --steps 200 --warmup 20
b ocp_rows_b1 --ocp rows --batch 1 --steps 30 --warmup 3
b ocp_projected_b4096 --ocp projected --steps 20 --warmup 3
b ocp_rows_b4096 --ocp rows --steps 10 --warmup 2
cd /tmp && export TMPDIR=/tmp
[ -z "$ONLY_OCP" ] && { timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --cpu-sample 0 > $O/prof.log 2>&1; rc=$?; fatal $rc prof; [ $rc -ne 0 ] && exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_ocp_p1 -o run --output-format csv -- python3 $R/bench.py --ocp projected --batch 1 --steps 100 --warmup 10 --cpu-sample 0 --no-tick > $O/prof_ocp_p1.log 2>&1; rc=$?; fatal $rc prof_ocp_p1; [ $rc -ne 0 ] && exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_ocp_r1 -o run --output-format csv -- python3 $R/bench.py --ocp rows --batch 1 --steps 20 --warmup 2 --cpu-sample 0 --no-tick > $O/prof_ocp_r1.log 2>&1; rc=$?; fatal $rc prof_ocp_r1; [ $rc -ne 0 ] && exit 1
echo all_done
