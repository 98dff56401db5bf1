#!/bin/bash
# Session script: SQP step with 5 stored CoM paths (tests + NLP A/B vs base), k_ipm72 phase stamps.
O=gpurun_out/r04p; mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_feet.py tests/test_sqp.py tests/test_ipm72.py tests/test_reference_nlp.py -m gpu > $O/pytest.log 2>&1; rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
nlp() { CMPC_LIB=$2 timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --sqp-iters 10 --nlp --no-e2e --cpu-sample 0 $3 > $O/nlp_$1.json 2>$O/nlp_$1.err || exit 9; python3 -c "import json;d=json.load(open('$O/nlp_$1.json'));print('$1',round(d['value']),round(d['ms_per_step'],4),d['solver'])"; }
for i in 1 2; do
  nlp new$i cheeta-mpc_amd/lib/libcmpc.so
  nlp base$i lab/_ab/libcmpc_base.so
done
CMPC_LIB=lab/_stamps/libcmpc_ipm72stamps.so timeout -k 10 200 python -u lab/ipm72_stamps.py > $O/stamps.log 2>&1; rc=$?; cat $O/stamps.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_nlp -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --cpu-sample 0 --steps 5 --warmup 1 --sqp-iters 10 --nlp --no-e2e > $GRAFT_REPO_ROOT/$O/prof_nlp.log 2>&1; echo "prof rc $?"
