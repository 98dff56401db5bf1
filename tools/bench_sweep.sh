#!/bin/bash
# GPU-box script: bench every BASELINE config that fits one GPU (+ the large size class), one JSON line each,
# and a rocprofv3 kernel-stats pass of the all-stance N=20 run. Stops at the first failing step.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O
cd $R
run() { name=$1; shift; timeout -k 10 240 python bench.py --cpu-sample 0 "$@" > $O/sweep_$name.json 2> $O/sweep_$name.err || { echo "FAIL $name rc=$?"; tail -5 $O/sweep_$name.err; exit 1; }; echo "$name $(cat $O/sweep_$name.json)"; }
run c2_trot_n10_f64
run c3_trot_n20_f32 --horizon 20 --precision f32
run c3_trot_n20_f64 --horizon 20
run c5_mixed_n10_f64 --gait 1
run pronk_n20_f64 --horizon 20 --all-stance
run pronk_n20_f32 --horizon 20 --all-stance --precision f32
run c4_shard_b32768 --batch 32768
run sqp_mixed_n10_f64 --gait 1 --sqp-iters 10 --steps 5
run sqp_trot_n10_f64 --sqp-iters 10 --steps 5
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_pronk -o run --output-format csv -- python3 $R/bench.py --horizon 20 --all-stance --steps 5 --cpu-sample 0 > $O/prof_pronk.log 2>&1 || { echo "prof fail"; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_mixed -o run --output-format csv -- python3 $R/bench.py --gait 1 --steps 10 --cpu-sample 0 > $O/prof_mixed.log 2>&1 || { echo "prof fail"; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof_n20f32 -o run --output-format csv -- python3 $R/bench.py --horizon 20 --precision f32 --steps 10 --cpu-sample 0 > $O/prof_n20f32.log 2>&1 || { echo "prof fail"; exit 1; }
echo sweep_done
