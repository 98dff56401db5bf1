#!/bin/bash
# Session script: SQP / NLP tests on the restructured k_sqp_step, NLP stamps (k_sqp_step, foothold condensing).
O=gpurun_out/r04z; mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_feet.py tests/test_sqp.py tests/test_ipm72.py tests/test_reference_nlp.py -m gpu > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
CMPC_LIB=lab/_stamps/libcmpc_nlpstamps.so timeout -k 10 200 python -u lab/nlp_stamps.py > $O/stamps.log 2>&1; rc=$?; cat $O/stamps.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --sqp-iters 10 --nlp --no-e2e --cpu-sample 0 > $O/nlp.json 2>$O/nlp.err || exit 9; python3 -c "import json;d=json.load(open('$O/nlp.json'));print('nlp',round(d['value']),round(d['ms_per_step'],4))"
timeout -k 10 200 env CMPC_LIB=lab/_ab/libcmpc_prev.so python -u bench.py --steps 20 --warmup 3 --sqp-iters 10 --nlp --no-e2e --cpu-sample 0 > $O/nlp_prev.json 2>$O/nlp_prev.err || exit 9; python3 -c "import json;d=json.load(open('$O/nlp_prev.json'));print('nlp_prev',round(d['value']),round(d['ms_per_step'],4))"
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --sqp-iters 10 --no-e2e --cpu-sample 0 > $O/sqp.json 2>$O/sqp.err || exit 9; python3 -c "import json;d=json.load(open('$O/sqp.json'));print('sqp_frozen',round(d['value']),round(d['ms_per_step'],4))"
timeout -k 10 200 env CMPC_LIB=lab/_ab/libcmpc_prev.so python -u bench.py --steps 20 --warmup 3 --sqp-iters 10 --no-e2e --cpu-sample 0 > $O/sqp_prev.json 2>$O/sqp_prev.err || exit 9; python3 -c "import json;d=json.load(open('$O/sqp_prev.json'));print('sqp_frozen_prev',round(d['value']),round(d['ms_per_step'],4))"
