#!/bin/bash
# GPU-box script: FETCH_SIZE / WRITE_SIZE passes (separate) of one bench command -> gpurun_out/traffic_<key>.json,
# keyed by bench.py's workload key and stamped with the libcmpc.so md5 (copy it to profiles/ to have bench.py report
# roofline.traffic for that workload). BENCH_ARGS / KEY pick the workload.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/traffic_${KEY:-N10_B4096_f64_trot}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --stats -d $O/pmc_$c -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-sample 0 ${BENCH_ARGS:-} > $O/pmc_$c.log 2>&1; rc=$?
  echo "pmc_$c rc=$rc"; [ $rc -ne 0 ] && exit 1
done
python3 $R/cheeta-mpc_amd/tools/pmc_traffic.py $O $R/gpurun_out/traffic_${KEY:-N10_B4096_f64_trot}.json "${BENCH_ARGS:-}"
