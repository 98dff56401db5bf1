#!/bin/bash
# GPU-box script: GPU tests, then A/B of the in-tree libcmpc.so against lab/build/libcmpc_old.so (CMPC_LIB) on the
# headline and configs 3 / 5, then FETCH_SIZE / WRITE_SIZE traffic of the in-tree build for the three workloads.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/h64; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -2 $O/gpu_tests.log; [ $rc -ne 0 ] && exit 1
for r in 1 2; do
 for W in ${AB_SET:-"c2|" "c3|--horizon 20 --precision f32" "c5|--gait 1"}; do
  L=${W%%|*}; BA=${W#*|}
  for V in new old; do
   if [ $V = old ]; then export CMPC_LIB=$R/lab/build/libcmpc_old.so; else unset CMPC_LIB; fi
   timeout -k 10 200 python bench.py --cpu-sample 0 --no-e2e --steps 100 $BA > $O/${L}_${V}_$r.json 2>$O/${L}_${V}_$r.err || exit 1
   python3 -c "import json;d=json.load(open('$O/${L}_${V}_$r.json'));print('$L $V',$r,round(d['value']),{k: round(v,4) for k,v in d['stages_ms'].items()})"
  done
 done
done
unset CMPC_LIB
cd /tmp && export TMPDIR=/tmp
for W in "N10_B4096_f64_trot|" "N20_B4096_f32_trot|--horizon 20 --precision f32" "N10_B4096_f64_mixed|--gait 1"; do
  KEY=${W%%|*}; BA=${W#*|}; D=$O/traffic_$KEY; mkdir -p $D
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --stats -d $D/pmc_$c -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-sample 0 $BA > $D/pmc_$c.log 2>&1 || exit 1
  done
  python3 $R/cheeta-mpc_amd/tools/pmc_traffic.py $D $O/traffic_$KEY.json "$BA" > $D/summary.txt && echo $KEY && cat $D/summary.txt
done
