#!/bin/bash
# GPU-box script: the bordered n = 66 class (k_ipm72): its tests and the NLP / QP suites, then NLP bench lines
# with CMPC_PATH_IPM72 on / off and config 5 / headline against lab/prev/libcmpc_old.so (the build before).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/ipm72; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_ipm72.py -x -v --timeout 120 --timeout-method thread > $O/t72.log 2>&1; rc=$?
tail -15 $O/t72.log; [ $rc -ne 0 ] && exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log; [ $rc -ne 0 ] && exit 1
for r in 1 2; do
  for A in "nlp72|--sqp-iters 10 --nlp --steps 20 --warmup 5" "nlp128|--sqp-iters 10 --nlp --steps 20 --warmup 5 --path IPM72=0"; do
    L=${A%%|*}; BA=${A#*|}
    timeout -k 10 200 python bench.py --cpu-sample 0 $BA > $O/${L}_$r.json 2> $O/${L}_$r.err || { tail -5 $O/${L}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${L}_$r.json'));print('$L',$r,round(d['value']),d['ms_per_step'])"
  done
  for W in "c5|--gait 1" "c2|"; do
    L=${W%%|*}; BA=${W#*|}
    for V in new old; do
      if [ $V = old ]; then export CMPC_LIB=$R/lab/prev/libcmpc_old.so; else unset CMPC_LIB; fi
      timeout -k 10 200 python bench.py --cpu-sample 0 --no-e2e --steps 100 $BA > $O/${L}_${V}_$r.json 2>$O/${L}_${V}_$r.err || exit 1
      python3 -c "import json;d=json.load(open('$O/${L}_${V}_$r.json'));print('$L $V',$r,round(d['value']),{k: round(v,4) for k,v in d['stages_ms'].items()})"
    done
    unset CMPC_LIB
  done
done
