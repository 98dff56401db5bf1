#!/bin/bash
# GPU-box script: rocprofv3 counter passes over one bench.py command (one pass per argument, counters space-separated
# inside the argument; each pass within the per-block slot limits of MI355X_MICROARCH.md). BENCH_ARGS picks the
# workload (default: the headline). Every pass has its own hard time limit; a failed pass ends the script.
#   bash tools/gpu_pmc.sh "SQ_WAVES SQ_INSTS_VALU" "FETCH_SIZE" ...
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/pmc; mkdir -p $O
BA=${BENCH_ARGS:-"--steps 3 --warmup 1 --cpu-sample 0"}
cd /tmp && export TMPDIR=/tmp
if [ "${LIST:-0}" = "1" ]; then timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1; echo "list rc=$?"; fi
i=0
for P in "$@"; do
  i=$((i+1))
  if [ -s $O/counters.txt ]; then
    miss=""; for c in $P; do grep -qw "$c" $O/counters.txt || miss="$miss $c"; done
    [ -n "$miss" ] && { echo "pass $i skipped: not listed:$miss"; continue; }
  fi
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --stats -d $O/p$i -o run --output-format csv -- python3 $R/bench.py $BA > $O/p$i.log 2>&1; rc=$?
  echo "pass $i ($P) rc=$rc"
  [ $rc -ne 0 ] && { tail -5 $O/p$i.log; exit 1; }
done
python3 $R/cheeta-mpc_amd/tools/pmc_summary.py $O > $O/summary.txt && cat $O/summary.txt
echo all_done
