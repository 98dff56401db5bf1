#!/bin/bash
# GPU-box script (round 4 final evidence, re-entry session): GPU tests, smoke, headline bench with the CPU baseline, configs 3 / 5, NLP, the
# OCP bench lines (projected / rows, with the CPU oracle), rocprofv3 kernel stats of the headline and of B = 1 OCP
# solves, FETCH_SIZE / WRITE_SIZE traffic and SQ counter passes for the headline and configs 3 / 5 (md5-stamped).
# Every GPU step has its own time limit; a fault / abort / time-out ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/final5; mkdir -p $O; cd $R
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; fatal $rc tests
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; fatal $rc smoke
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?; echo bench_rc=$rc; fatal $rc bench
python3 -c "import json;d=json.load(open('$O/bench.json'));print(round(d['value']),d['stages_ms'],d['roofline']['frac'],d['cpu_baseline']['value'])"
b() { local n=$1; shift; timeout -k 10 300 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err; local rc=$?; fatal $rc $n
      python3 -c "import json;d=json.loads(open('$O/$n.json').read().strip().split(chr(10))[-1]);print('$n',round(d['value']),d['unit'],round(d['ms_per_step'],4),d.get('stages_ms'),d.get('ms_per_solve_b1'),d['roofline']['frac'])" || tail -3 $O/$n.err; }
b c3 --horizon 20 --precision f32 --steps 100 --warmup 20 --cpu-sample 0
b c5 --gait 1 --steps 100 --warmup 20 --cpu-sample 0
b nlp_trot --steps 20 --warmup 3 --sqp-iters 10 --nlp --no-e2e --cpu-sample 0
b sqp_trot --steps 20 --warmup 3 --sqp-iters 10 --no-e2e --cpu-sample 0
b drv --steps 20 --warmup 5
b ocp_projected --ocp projected --steps 20 --warmup 3
b ocp_rows --ocp rows --steps 10 --warmup 2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --cpu-sample 0 > $O/prof.log 2>&1; rc=$?; fatal $rc prof; [ $rc -ne 0 ] && exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_ocp_b1 -o run --output-format csv -- python3 $R/tools/ocp_probe.py 1 > $O/prof_ocp_b1.log 2>&1; rc=$?; fatal $rc prof_ocp; [ $rc -ne 0 ] && exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_nlp -o run --output-format csv -- python3 $R/bench.py --cpu-sample 0 --steps 5 --warmup 1 --sqp-iters 10 --nlp --no-e2e > $O/prof_nlp.log 2>&1; rc=$?; fatal $rc prof_nlp; [ $rc -ne 0 ] && exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o run --output-format csv -- python3 $R/bench.py --cpu-sample 0 --steps 20 --gait 1 > $O/prof_c5.log 2>&1; rc=$?; fatal $rc prof_c5; [ $rc -ne 0 ] && exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python3 $R/bench.py --cpu-sample 0 --steps 20 --horizon 20 --precision f32 > $O/prof_c3.log 2>&1; rc=$?; fatal $rc prof_c3; [ $rc -ne 0 ] && exit 1
for W in "N10_B4096_f64_trot|" "N20_B4096_f32_trot|--horizon 20 --precision f32" "N10_B4096_f64_mixed|--gait 1"; do
  KEY=${W%%|*}; BA=${W#*|}; D=$O/traffic_$KEY; mkdir -p $D
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --stats -d $D/pmc_$c -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-sample 0 $BA > $D/pmc_$c.log 2>&1; rc=$?
    echo "$KEY $c rc=$rc"; [ $rc -ne 0 ] && exit 1
  done
  python3 $R/cheeta-mpc_amd/tools/pmc_traffic.py $D $O/traffic_$KEY.json "$BA" > $D/summary.txt || exit 1
done
for W in "head|N10_B4096_f64_trot|" "c3|N20_B4096_f32_trot|--horizon 20 --precision f32" "c5|N10_B4096_f64_mixed|--gait 1"; do
  KEY=${W%%|*}; R2=${W#*|}; WK=${R2%%|*}; BA=${R2#*|}; D=$O/sq_$KEY; mkdir -p $D; i=0
  for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT" "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --stats -d $D/p$i -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-sample 0 $BA > $D/p$i.log 2>&1; rc=$?
    echo "sq $KEY pass $i rc=$rc"; [ $rc -ne 0 ] && exit 1
  done
  python3 $R/cheeta-mpc_amd/tools/pmc_summary.py $D --json $O/pmc_sq_$WK.json > $O/sq_$KEY.txt || exit 1
done
echo all_done
