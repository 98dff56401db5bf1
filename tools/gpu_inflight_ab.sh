#!/bin/bash
# A/B of the batch-level pipeline depth (bench.py --inflight K) on the headline workload, alternating K twice.
set -o pipefail
out=gpurun_out/inflight
mkdir -p $out
for rep in 1 2; do
  for k in 1 2 3 4; do
    timeout -k 10 120 python -u bench.py --inflight $k --cpu-sample 0 --no-e2e --steps 40 --warmup 10 \
      > $out/k${k}_r${rep}.json 2> $out/k${k}_r${rep}.err || exit $?
  done
done
