#!/bin/bash
# GPU-box script: the driver's round-end sequence (pytest -m gpu -x, smoke), then the headline bench (with the
# end-to-end gather pass) and the self-launched two-rank bench on the box's one GPU. Every GPU step has its own time
# limit; a failure, fault or time-out ends the script (no further GPU step).
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/check; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print(round(d['value']),round(d['value_end_to_end'] or 0),d['gather'],d['stages_ms'],d['roofline']['frac'],d['cpu_baseline']['value'],d['build'])"
timeout -k 10 300 python bench.py --gpus 2 --cpu-sample 0 > $O/bench2.json 2> $O/bench2.err || { tail $O/bench2.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench2.json'));print(d['n_gpus'],round(d['value']),round(d['value_end_to_end'] or 0),d['gather'])"
