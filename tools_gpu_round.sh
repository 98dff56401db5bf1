#!/bin/bash
# GPU-box script: tests, smoke, bench, rocprofv3 kernel stats and HBM counters (each step under its own timeout).
set -o pipefail
R=$GRAFT_REPO_ROOT; [ -z "$R" ] && R=$(pwd)
O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 400 python -m pytest tests -m gpu -q > $O/gpu_tests.log 2>&1; echo "tests_exit=$?"; tail -4 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke_exit=$?"; tail -2 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --cpu-sample 0 > $O/prof.log 2>&1 || { echo prof failed; tail $O/prof.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --stats -d $O/pmc_$c -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --cpu-sample 0 > $O/pmc_$c.log 2>&1 || { echo pmc $c failed; tail $O/pmc_$c.log; exit 1; }
done
echo all_done
