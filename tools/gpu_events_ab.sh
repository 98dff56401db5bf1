#!/bin/bash
# A/B of the measurement overhead: stage events on every timed step (--event-frac 1), on the last quarter of them
# (default), after the timed region (--stage-events after), and hipGraph replay; headline workload, alternating 3 times.
set -o pipefail
out=gpurun_out/events2
mkdir -p $out
for rep in 1 2 3; do
  for v in "all:--event-frac 1" "quarter:" "after:--stage-events after" "graph:--graph 1"; do
    name=${v%%:*}; flags=${v#*:}
    timeout -k 10 120 python -u bench.py $flags --cpu-sample 0 --no-e2e --steps 60 --warmup 10 \
      > $out/${name}_r${rep}.json 2> $out/${name}_r${rep}.err || exit $?
  done
done
