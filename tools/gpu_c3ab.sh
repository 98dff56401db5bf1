#!/bin/bash
# GPU-box script: config 3 (N = 20 trot fp32) and config 5 bench lines, twice each, plus the 128-class parity tests.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/c3ab; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_class128.py tests/test_fused128.py tests/test_full_size.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || exit 1
for r in 1 2; do
for A in "c3|--horizon 20 --precision f32" "c5|--gait 1" "c2|"; do
  L=${A%%|*}; ARGS=${A#*|}
  timeout -k 10 200 python bench.py --cpu-sample 0 --no-e2e --steps 100 --warmup 20 $ARGS > $O/${L}_$r.json 2> $O/${L}_$r.err || { tail $O/${L}_$r.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/${L}_$r.json'));print('$L', $r, round(d['value']), {k: round(v,4) for k,v in d['stages_ms'].items()})"
done; done
