#!/bin/bash
# Session script: SQP staging from the LDS copies: SQP / NLP tests, stamps, NLP / SQP A/B against the previous build.
O=gpurun_out/r04ac; mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_feet.py tests/test_sqp.py tests/test_ipm72.py tests/test_reference_nlp.py tests/test_policy.py -m gpu > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
CMPC_LIB=lab/_stamps/libcmpc_nlpstamps.so timeout -k 10 200 python -u lab/nlp_stamps.py > $O/stamps.log 2>&1; rc=$?; head -18 $O/stamps.log; [ $rc -eq 0 ] || exit $rc
b() { n=$1; lib=$2; shift 2; CMPC_LIB=$lib timeout -k 10 300 python -u bench.py --cpu-sample 0 --no-e2e "$@" > $O/$n.json 2> $O/$n.err || exit 9
      python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',round(d['value']),round(d['ms_per_step'],4))"; }
for i in 1 2; do
  b nlp_new$i cheeta-mpc_amd/lib/libcmpc.so --steps 20 --warmup 3 --sqp-iters 10 --nlp
  b nlp_prev$i lab/_ab/libcmpc_prev.so --steps 20 --warmup 3 --sqp-iters 10 --nlp
  b sqp_new$i cheeta-mpc_amd/lib/libcmpc.so --steps 20 --warmup 3 --sqp-iters 10
  b sqp_prev$i lab/_ab/libcmpc_prev.so --steps 20 --warmup 3 --sqp-iters 10
done
