#!/bin/bash
# Session script (round 4 m, re-entry): the current build end to end — GPU tests, C++ mirror, smoke, headline /
# configs 3 / 5 / NLP / OCP bench lines, B = 1 OCP probe. Every GPU step has its own limit; a fatal exit ends it.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$R/gpurun_out/r04m; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1; rc=$?
echo "pytest rc $rc"; tail -6 $O/pytest.log; fatal $rc pytest
timeout -k 10 200 tests/cpp/bin/test_hpipm_interface > $O/cpp.log 2>&1; rc=$?; echo "cpp rc $rc"; tail -3 $O/cpp.log; fatal $rc cpp
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; fatal $rc smoke
b() { local n=$1; shift; timeout -k 10 300 python -u bench.py --cpu-sample 0 "$@" > $O/$n.json 2> $O/$n.err; local rc=$?; fatal $rc $n
      python3 -c "import json;d=json.loads(open('$O/$n.json').read().strip().split(chr(10))[-1]);print('$n',round(d['value']),d['unit'],round(d['ms_per_step'],4),d.get('stages_ms'),d.get('ms_per_solve_b1'),d['roofline']['frac'])" || tail -3 $O/$n.err; }
b drv --steps 20 --warmup 5
b head --steps 200 --warmup 50
b c5 --gait 1 --steps 100 --warmup 20
b c3 --horizon 20 --precision f32 --steps 100 --warmup 20
b nlp_trot --steps 20 --warmup 3 --sqp-iters 10 --nlp --no-e2e
b ocp_projected --ocp projected --steps 20 --warmup 3
b ocp_rows --ocp rows --steps 10 --warmup 2
timeout -k 10 200 python -u tools/ocp_probe.py 1 1024 > $O/probe.log 2>&1; rc=$?; cat $O/probe.log; fatal $rc probe
echo all_done
