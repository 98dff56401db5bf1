#!/bin/bash
# GPU-box script: k_ric parity tests, phase stamps (lab build), and bench lines of the stage-wise path.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/ricq; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_ric.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -4 $O/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python lab/ric_stamps.py || exit 1
for A in "c2_ric2|--ric 2" "c5_ric1|--gait 1 --ric 1" "c3_ric1|--horizon 20 --precision f32 --ric 1"; do
  L=${A%%|*}; ARGS=${A#*|}
  timeout -k 10 200 python bench.py --cpu-sample 0 --no-e2e --steps 50 --warmup 10 $ARGS > $O/$L.json 2> $O/$L.err || { tail $O/$L.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$L.json'));print('$L', round(d['value']), {k: round(v,4) for k,v in d['stages_ms'].items()})"
done
