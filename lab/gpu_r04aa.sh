#!/bin/bash
# Session script: the whole GPU suite, smoke, C++ mirror and the driver's headline command on the current build.
O=gpurun_out/r04aa; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1; rc=$?
echo "pytest rc $rc"; tail -4 $O/pytest.log; fatal $rc pytest; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 tests/cpp/bin/test_hpipm_interface > $O/cpp.log 2>&1; rc=$?; echo "cpp rc $rc"; tail -2 $O/cpp.log; fatal $rc cpp
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; fatal $rc smoke
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/drv.json 2> $O/drv.err; rc=$?; fatal $rc bench
python3 -c "import json;d=json.load(open('$O/drv.json'));print('drv',round(d['value']),d['warmup_run'],d['stages_ms'],d['roofline']['frac'],d['roofline']['traffic'],d['cpu_baseline']['value'])"
