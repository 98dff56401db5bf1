#!/bin/bash
# Session script: OCP staged residual vectors, k_ipm72 forward-only Schur, 80-row H block for k_ipm72's QPs:
# tests and same-box A/B (new / h72 = old k_ipm72 / old = old k_ipm72 + old condensing).
O=gpurun_out/r04l; mkdir -p $O
t() { timeout -k 10 "$@"; }
t 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_ocp_ipm.py tests/test_ocp_eq.py tests/test_ipm72.py tests/test_feet.py tests/test_sqp.py -m gpu > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
nlp() { CMPC_LIB=$2 t 200 python -u bench.py --steps 20 --warmup 3 --sqp-iters 10 --nlp --no-e2e --cpu-sample 0 > $O/nlp_$1.json 2>$O/nlp_$1.err || exit 9; python3 -c "import json;d=json.load(open('$O/nlp_$1.json'));print('$1',d['value'],d['ms_per_step'])"; }
for i in 1 2; do
  t 200 python -u tools/ocp_probe.py 1 1024 > $O/probe$i.log 2>&1 || exit 9; cat $O/probe$i.log
  CMPC_LIB=lab/_ab/libcmpc_prev.so t 200 python -u tools/ocp_probe.py 1 1024 > $O/probe_prev$i.log 2>&1 || exit 9; cat $O/probe_prev$i.log
  nlp new$i cheeta-mpc_amd/lib/libcmpc.so
  nlp h72_$i lab/_ab/libcmpc_h72.so
  nlp old$i lab/_ab/libcmpc_old.so
done
CMPC_LIB=lab/_stamps/libcmpc_ocpstamps.so t 200 python -u tools/ocp_probe.py --stamps > $O/stamps.log 2>&1; cat $O/stamps.log
