#!/bin/bash
# GPU-box script for the lab harness: variant timings + stamps, then counter passes on the product variant.
# Every GPU step has its own timeout; a fault/abort/timeout ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/lab; mkdir -p $O
cd $R
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
LAB_OUT=$O timeout -k 10 240 ./lab/ipm_lab ${LAB_B:-4096} 25 > $O/lab.json 2> $O/lab.err; rc=$?; echo "lab rc=$rc"; cat $O/lab.json; fatal $rc lab
[ $rc -ne 0 ] && exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1; echo "list rc=$?"
i=0
for P in "$@"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $P --kernel-trace --stats -d $O/pmc$i -o run --output-format csv -- $R/lab/ipm_lab 4096 2 v0_prod > $O/pmc$i.log 2>&1; rc=$?
  echo "pmc$i ($P) rc=$rc"; fatal $rc pmc$i
done
echo all_done
