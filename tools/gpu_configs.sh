#!/bin/bash
# GPU-box script: bench lines for the BASELINE configs besides the headline (config 3: N=20 trot fp32; config 5:
# mixed gait; config 4 share: B=32768) and the all-stance classes, then kernel stats of configs 3 and 5.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/cfg; mkdir -p $O; cd $R
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
run() { name=$1; shift; timeout -k 10 200 python bench.py --cpu-sample 0 "$@" > $O/$name.json 2> $O/$name.err; rc=$?; fatal $rc $name; [ $rc -ne 0 ] && { tail -3 $O/$name.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$name.json'));print('$name',round(d['value']),{k:round(v,4) for k,v in d['stages_ms'].items()},round(d['roofline']['frac'],4))"; }
run c3 --horizon 20 --precision f32
run c5 --gait 1
run c4share --batch 32768 --steps 5
run pronk10 --all-stance
[ "${PROF:-1}" = "0" ] && exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python3 $R/bench.py --steps 10 --cpu-sample 0 --horizon 20 --precision f32 > $O/prof_c3.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o run --output-format csv -- python3 $R/bench.py --steps 10 --cpu-sample 0 --gait 1 > $O/prof_c5.log 2>&1 || exit 1
for c in c3 c5; do echo $c; cut -d, -f1-4 $O/prof_$c/run_kernel_stats.csv | head -7; done
