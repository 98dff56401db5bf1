#!/bin/bash
# Session script: k_ipm72 GJ pivots and border exchanges by readlane: tests, stamps, NLP A/B.
O=gpurun_out/r04t; mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_feet.py tests/test_sqp.py tests/test_ipm72.py tests/test_reference_nlp.py -m gpu > $O/pytest.log 2>&1; rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
CMPC_LIB=lab/_stamps/libcmpc_ipm72stamps.so timeout -k 10 200 python -u lab/ipm72_stamps.py > $O/stamps.log 2>&1; rc=$?; cat $O/stamps.log; [ $rc -eq 0 ] || exit $rc
nlp() { CMPC_LIB=$2 timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --sqp-iters 10 --nlp --no-e2e --cpu-sample 0 $3 > $O/nlp_$1.json 2>$O/nlp_$1.err || exit 9; python3 -c "import json;d=json.load(open('$O/nlp_$1.json'));print('$1',round(d['value']),round(d['ms_per_step'],4),d['solver'])"; }
for i in 1 2; do
  nlp new$i cheeta-mpc_amd/lib/libcmpc.so
  nlp prev$i lab/_ab/libcmpc_prev.so
done
