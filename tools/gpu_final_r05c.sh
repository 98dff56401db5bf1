#!/bin/bash
# GPU-box script (round 5 final evidence, part C): the bench lines again once the md5-stamped counter summaries of this
# build are in profiles/ (their roofline.traffic / sq_counters are then filled in).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/final_r05c; mkdir -p $O; cd $R
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
b() { local n=$1; shift; timeout -k 10 300 python -u bench.py "$@" > $O/$n.json 2> $O/$n.err; local rc=$?; fatal $rc $n
      python3 -c "import json;d=json.loads(open('$O/$n.json').read().strip().split(chr(10))[-1]);print('$n',round(d['value']),d['ms_per_step'],d['roofline']['traffic'],d['roofline']['frac'])" || tail -3 $O/$n.err; }
b bench --cadence 20
b ocp_projected_b1 --ocp projected --batch 1 --steps 200 --warmup 20
b ocp_rows_b1 --ocp rows --batch 1 --steps 30 --warmup 3
b ocp_projected_b4096 --ocp projected --steps 20 --warmup 3
b ocp_rows_b4096 --ocp rows --steps 10 --warmup 2
echo all_done
