#!/bin/bash
# GPU-box script: the headline bench under several environments, alternating rounds (no tests).
#   AB="label1=ENV=V ENV2=W;label2=...;..." ROUNDS=2 bash tools_gpu_abenv.sh
# a failing step ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
IFS=';' read -ra CASES <<< "$AB"
for r in $(seq 1 ${ROUNDS:-2}); do
  for c in "${CASES[@]}"; do
    lab=${c%%=*}; envs=${c#*=}
    env $envs timeout -k 10 200 python bench.py --cpu-sample 0 ${BENCH_ARGS:-} > $O/ab_$lab.json 2> $O/ab_$lab.err; rc=$?
    fatal $rc "$lab"; [ $rc -ne 0 ] && { tail -3 $O/ab_$lab.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/ab_$lab.json'));print('$lab',round(d['value']),{k:round(v,4) for k,v in d['stages_ms'].items()},round(d['ms_per_step'],4))"
  done
done
