#!/bin/bash
# Session script: SQP staging in chunks + k_sqp_step occupancy (launch bounds 2 / 3 / 4 waves per SIMD): SQP / NLP
# tests on each, NLP / SQP A/B against the final-evidence build.
O=gpurun_out/r04ag; mkdir -p $O
for L in cur:cheeta-mpc_amd/lib/libcmpc.so w3:lab/_ab/libcmpc_w3.so w4:lab/_ab/libcmpc_w4.so; do
  n=${L%%:*}; CMPC_LIB=${L#*:} timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_feet.py tests/test_sqp.py tests/test_policy.py tests/test_reference_nlp.py -m gpu > $O/pytest_$n.log 2>&1; rc=$?; echo "$n $(tail -1 $O/pytest_$n.log)"; [ $rc -eq 0 ] || exit $rc
done
b() { n=$1; lib=$2; shift 2; CMPC_LIB=$lib timeout -k 10 300 python -u bench.py --cpu-sample 0 --no-e2e "$@" > $O/$n.json 2> $O/$n.err || exit 9
      python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',round(d['value']),round(d['ms_per_step'],4))"; }
for i in 1 2; do
  for L in cur:cheeta-mpc_amd/lib/libcmpc.so w3:lab/_ab/libcmpc_w3.so w4:lab/_ab/libcmpc_w4.so prev:lab/_ab/libcmpc_prev.so; do
    n=${L%%:*}; b nlp_$n$i ${L#*:} --steps 20 --warmup 3 --sqp-iters 10 --nlp
    b sqp_$n$i ${L#*:} --steps 20 --warmup 3 --sqp-iters 10
  done
done
