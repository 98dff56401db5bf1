#!/bin/bash
# Session script: coalesced mirror writes in the condensing epilogue: whole GPU suite, NLP stamps, A/B of NLP /
# config 3 / config 5 against the previous build.
O=gpurun_out/r04ab; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1; rc=$?
echo "pytest rc $rc"; tail -2 $O/pytest.log; fatal $rc pytest; [ $rc -eq 0 ] || exit 1
CMPC_LIB=lab/_stamps/libcmpc_nlpstamps.so timeout -k 10 200 python -u lab/nlp_stamps.py > $O/stamps.log 2>&1; rc=$?; grep -A9 condense80 $O/stamps.log; [ $rc -eq 0 ] || exit $rc
b() { n=$1; lib=$2; shift 2; CMPC_LIB=$lib timeout -k 10 300 python -u bench.py --cpu-sample 0 --no-e2e "$@" > $O/$n.json 2> $O/$n.err || exit 9
      python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',round(d['value']),round(d['ms_per_step'],4),d.get('stages_ms'))"; }
for i in 1 2; do
  b nlp_new$i cheeta-mpc_amd/lib/libcmpc.so --steps 20 --warmup 3 --sqp-iters 10 --nlp
  b nlp_prev$i lab/_ab/libcmpc_prev.so --steps 20 --warmup 3 --sqp-iters 10 --nlp
  b c5_new$i cheeta-mpc_amd/lib/libcmpc.so --gait 1 --steps 100 --warmup 20
  b c5_prev$i lab/_ab/libcmpc_prev.so --gait 1 --steps 100 --warmup 20
  b c3_new$i cheeta-mpc_amd/lib/libcmpc.so --horizon 20 --precision f32 --steps 100 --warmup 20
  b c3_prev$i lab/_ab/libcmpc_prev.so --horizon 20 --precision f32 --steps 100 --warmup 20
done
