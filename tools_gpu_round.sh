#!/bin/bash
# GPU-box script: tests, smoke, bench, rocprofv3 kernel stats and HBM counters. Each GPU step has its own timeout;
# a fault / abort / timeout ends the script (no further GPU step).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out; mkdir -p $O
cd $R
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 400 python -m pytest tests -m gpu -q > $O/gpu_tests.log 2>&1; rc=$?; echo "tests_exit=$rc"; tail -4 $O/gpu_tests.log; fatal $rc tests
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke_exit=$rc"; tail -2 $O/smoke.log; fatal $rc smoke
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?; echo "bench_exit=$rc"; cat $O/bench.json; fatal $rc bench
[ "${1:-}" = "noprof" ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --cpu-sample 0 > $O/prof.log 2>&1; rc=$?; echo "prof_exit=$rc"; fatal $rc prof
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --stats -d $O/pmc_$c -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-sample 0 > $O/pmc_$c.log 2>&1; rc=$?; echo "pmc_$c exit=$rc"; fatal $rc pmc_$c
done
python3 $R/cheeta-mpc_amd/tools/pmc_traffic.py $O $O/traffic.json && echo all_done
