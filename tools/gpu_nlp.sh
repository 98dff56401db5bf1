#!/bin/bash
# GPU-box script: NLP (footholds as variables) and frozen-foothold SQP throughput next to the headline QP, B = 4096.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/nlp; mkdir -p $O; cd $R
run() { timeout -k 10 200 python bench.py --cpu-sample 0 --no-e2e "$@"; }
run --steps 100 --warmup 20 > $O/qp.json 2> $O/qp.err || { tail $O/qp.err; exit 1; }
run --steps 20 --warmup 3 --sqp-iters 10 > $O/sqp_trot.json 2> $O/sqp_trot.err || { tail $O/sqp_trot.err; exit 1; }
run --steps 20 --warmup 3 --sqp-iters 10 --nlp > $O/nlp_trot.json 2> $O/nlp_trot.err || { tail $O/nlp_trot.err; exit 1; }
run --steps 20 --warmup 3 --sqp-iters 10 --gait 1 > $O/sqp_mixed.json 2> $O/sqp_mixed.err || { tail $O/sqp_mixed.err; exit 1; }
run --steps 20 --warmup 3 --sqp-iters 10 --nlp --gait 1 > $O/nlp_mixed.json 2> $O/nlp_mixed.err || { tail $O/nlp_mixed.err; exit 1; }
for f in qp sqp_trot nlp_trot sqp_mixed nlp_mixed; do
  python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f',round(d['value']),d['unit'],round(d['ms_per_step'],3),d['solver'])"
done
