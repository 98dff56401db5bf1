#!/bin/bash
# Session script: OCP unrolled stage-parallel loops + condensing lin / Q_k prefetch: whole GPU suite, A/B (NLP, SQP,
# configs 3 / 5, headline, OCP probe) against the final-evidence build.
O=gpurun_out/r04ae; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1; rc=$?
echo "pytest rc $rc"; tail -2 $O/pytest.log; fatal $rc pytest; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 tests/cpp/bin/test_hpipm_interface > $O/cpp.log 2>&1; rc=$?; echo "cpp rc $rc"; fatal $rc cpp
b() { n=$1; lib=$2; shift 2; CMPC_LIB=$lib timeout -k 10 300 python -u bench.py --cpu-sample 0 --no-e2e "$@" > $O/$n.json 2> $O/$n.err || exit 9
      python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',round(d['value']),round(d['ms_per_step'],4))"; }
for i in 1 2; do
  b nlp_new$i cheeta-mpc_amd/lib/libcmpc.so --steps 20 --warmup 3 --sqp-iters 10 --nlp
  b nlp_prev$i lab/_ab/libcmpc_prev.so --steps 20 --warmup 3 --sqp-iters 10 --nlp
  b sqp_new$i cheeta-mpc_amd/lib/libcmpc.so --steps 20 --warmup 3 --sqp-iters 10
  b sqp_prev$i lab/_ab/libcmpc_prev.so --steps 20 --warmup 3 --sqp-iters 10
  b c5_new$i cheeta-mpc_amd/lib/libcmpc.so --gait 1 --steps 100 --warmup 20
  b c5_prev$i lab/_ab/libcmpc_prev.so --gait 1 --steps 100 --warmup 20
  b c3_new$i cheeta-mpc_amd/lib/libcmpc.so --horizon 20 --precision f32 --steps 100 --warmup 20
  b c3_prev$i lab/_ab/libcmpc_prev.so --horizon 20 --precision f32 --steps 100 --warmup 20
done
export OCP_REPS=20
for L in new:cheeta-mpc_amd/lib/libcmpc.so prev:lab/_ab/libcmpc_prev.so new2:cheeta-mpc_amd/lib/libcmpc.so prev2:lab/_ab/libcmpc_prev.so; do
  n=${L%%:*}; CMPC_LIB=${L#*:} timeout -k 10 200 python -u tools/ocp_probe.py 1 1024 > $O/ocp_$n.log 2>&1 || { cat $O/ocp_$n.log; exit 9; }
  sed "s/^/$n /" $O/ocp_$n.log
done
