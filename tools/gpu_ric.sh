#!/bin/bash
# GPU-box script: stage-wise (Riccati) path parity tests, then bench A/B of the condensed vs stage-wise paths on
# configs 2, 5 and 3. Every GPU step has its own time limit; a failure ends the script.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/ric; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_ric.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -25 $O/tests.log
[ $rc -eq 0 ] || [ "$RIC_BENCH_ANYWAY" = 1 ] || exit 1
for A in "c2_base|" "c2_ric2|--ric 2" "c5_base|--gait 1" "c5_ric1|--gait 1 --ric 1" "c5_ric2|--gait 1 --ric 2" \
         "c3_base|--horizon 20 --precision f32" "c3_ric1|--horizon 20 --precision f32 --ric 1" "c3_ric2|--horizon 20 --precision f32 --ric 2"; do
  L=${A%%|*}; ARGS=${A#*|}
  timeout -k 10 200 python bench.py --cpu-sample 0 --no-e2e --steps 50 --warmup 10 $ARGS > $O/$L.json 2> $O/$L.err || { tail $O/$L.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$L.json'));print('$L', round(d['value']), {k: round(v,4) for k,v in d['stages_ms'].items()}, d['solver'])"
done
