#!/bin/bash
# GPU session script (round 4 e): full GPU tests, C++ mirror, benches (headline, configs 3 / 5, NLP), the OCP bench
# lines, rocprofv3 kernel stats of the NLP trot and of the OCP bench.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$R/gpurun_out/r04e; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1; rc=$?
echo "pytest rc $rc"; tail -6 $O/pytest.log; fatal $rc pytest
timeout -k 10 200 tests/cpp/bin/test_hpipm_interface > $O/cpp.log 2>&1; rc=$?; echo "cpp rc $rc"; tail -3 $O/cpp.log; fatal $rc cpp
b() { local n=$1; shift; timeout -k 10 300 python -u bench.py --cpu-sample 0 "$@" > $O/$n.json 2> $O/$n.err; local rc=$?; fatal $rc $n
      python3 -c "import json;d=json.loads(open('$O/$n.json').read().strip().split(chr(10))[-1]);print('$n',round(d['value']),d['unit'],round(d['ms_per_step'],4),d.get('stages_ms'),d.get('solver'))" || tail -3 $O/$n.err; }
b head --steps 200 --warmup 50
b c5 --gait 1 --steps 100 --warmup 20
b c3 --horizon 20 --precision f32 --steps 100 --warmup 20
b nlp_trot --steps 20 --warmup 3 --sqp-iters 10 --nlp --no-e2e
b nlp_mixed --steps 20 --warmup 3 --sqp-iters 10 --nlp --gait 1 --no-e2e
timeout -k 10 300 python -u bench.py --ocp projected --steps 20 --warmup 3 > $O/ocp_proj.json 2> $O/ocp_proj.err; rc=$?; fatal $rc ocp; tail -1 $O/ocp_proj.json | cut -c1-600; tail -3 $O/ocp_proj.err
timeout -k 10 300 python -u bench.py --ocp rows --steps 10 --warmup 2 > $O/ocp_rows.json 2> $O/ocp_rows.err; rc=$?; fatal $rc ocp; tail -1 $O/ocp_rows.json | cut -c1-600; tail -3 $O/ocp_rows.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_nlp -o run --output-format csv -- python3 $R/bench.py --cpu-sample 0 --steps 5 --warmup 1 --sqp-iters 10 --nlp --no-e2e > $O/prof_nlp.log 2>&1; rc=$?; echo "prof nlp rc $rc"; fatal $rc prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_ocp -o run --output-format csv -- python3 $R/bench.py --ocp rows --steps 5 --warmup 1 --cpu-sample 0 > $O/prof_ocp.log 2>&1; rc=$?; echo "prof ocp rc $rc"; fatal $rc prof
find $O -name "*kernel_stats.csv" | head
echo all_done
