#!/bin/bash
# GPU-box script (round 6 final evidence, part 2 of 2): GPU tests, smoke, the headline bench with the CPU baseline and
# the 50 Hz cadence line, configs 3 / 5, the OCP bench lines (projected / rows at B = 1 with the C++ mirror tick and
# its keep cost, and at B = 4096), rocprofv3 kernel stats of the headline, configs 3 / 5 and the B = 1 OCP solves, the
# OCP segment sweep. Run after gpu_final_r06b.sh with its summaries copied into profiles/ (same build). Every GPU step
# has its own time limit; a fault / abort / time-out ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/final_r06a; mkdir -p $O; cd $R
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; fatal $rc tests
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; fatal $rc smoke
fi
b() { local n=$1; shift; timeout -k 10 300 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err; local rc=$?; fatal $rc $n
      python3 -c "import json;d=json.loads(open('$O/$n.json').read().strip().split(chr(10))[-1]);t=d.get('tick') or {};print('$n',round(d['value']),d['unit'],round(d['ms_per_step'],4),d['roofline']['traffic'] if d.get('roofline') else None,d['roofline']['frac'] if d.get('roofline') else None,t.get('tick_ms_median'),t.get('keep_cost_ms_median'))" || tail -3 $O/$n.err; }
b bench --cadence 20
b c3 --horizon 20 --precision f32 --steps 100 --warmup 20 --cpu-sample 0
b c5 --gait 1 --steps 100 --warmup 20 --cpu-sample 0
b ocp_projected_b1 --ocp projected --batch 1 --steps 200 --warmup 20
b ocp_rows_b1 --ocp rows --batch 1 --steps 30 --warmup 3
b ocp_projected_b4096 --ocp projected --steps 20 --warmup 3
b ocp_rows_b4096 --ocp rows --steps 10 --warmup 2
for S in 1 4 6 8 10 12 14 16; do OCP_SEGS=$S timeout -k 10 120 python tools/ocp_probe.py 1 >> $O/ocp_segments.log 2>&1; rc=$?; fatal $rc probe; [ $rc -ne 0 ] && exit 1; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --cpu-sample 0 > $O/prof.log 2>&1; rc=$?; fatal $rc prof; [ $rc -ne 0 ] && exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python3 $R/bench.py --horizon 20 --precision f32 --steps 20 --cpu-sample 0 > $O/prof_c3.log 2>&1; rc=$?; fatal $rc prof_c3; [ $rc -ne 0 ] && exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o run --output-format csv -- python3 $R/bench.py --gait 1 --steps 20 --cpu-sample 0 > $O/prof_c5.log 2>&1; rc=$?; fatal $rc prof_c5; [ $rc -ne 0 ] && exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_ocp_p1 -o run --output-format csv -- python3 $R/bench.py --ocp projected --batch 1 --steps 100 --warmup 10 --cpu-sample 0 --no-tick > $O/prof_ocp_p1.log 2>&1; rc=$?; fatal $rc prof_ocp_p1; [ $rc -ne 0 ] && exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_ocp_r1 -o run --output-format csv -- python3 $R/bench.py --ocp rows --batch 1 --steps 20 --warmup 2 --cpu-sample 0 --no-tick > $O/prof_ocp_r1.log 2>&1; rc=$?; fatal $rc prof_ocp_r1; [ $rc -ne 0 ] && exit 1
echo all_done
