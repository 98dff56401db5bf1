#!/bin/bash
# GPU-box script: alternate bench.py argument sets for A/B measurement. Each argument is one set ("label|args").
#   bash tools/gpu_ab.sh "base|" "after|--stage-events after" ...   (ROUNDS=2 by default)
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/ab; mkdir -p $O; cd $R
ROUNDS=${ROUNDS:-2}
for r in $(seq 1 $ROUNDS); do
  for A in "$@"; do
    L=${A%%|*}; ARGS=${A#*|}
    timeout -k 10 200 python bench.py --cpu-sample 0 $ARGS > $O/${L}_$r.json 2> $O/${L}_$r.err || { tail $O/${L}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${L}_$r.json'));print('$L', $r, round(d['value']), round(d['value_end_to_end'] or 0), {k: round(v,4) for k,v in d['stages_ms'].items()})"
  done
done
