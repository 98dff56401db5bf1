#!/bin/bash
# A/B of hipGraph replay (bench.py --graph 1) against direct launches, headline and config 5, alternating twice.
set -o pipefail
out=gpurun_out/graph
mkdir -p $out
for rep in 1 2; do
  for g in 0 1; do
    timeout -k 10 120 python -u bench.py --graph $g --cpu-sample 0 --no-e2e --steps 40 --warmup 10 \
      > $out/c2_g${g}_r${rep}.json 2> $out/c2_g${g}_r${rep}.err || exit $?
    timeout -k 10 120 python -u bench.py --graph $g --gait 1 --cpu-sample 0 --no-e2e --steps 40 --warmup 10 \
      > $out/c5_g${g}_r${rep}.json 2> $out/c5_g${g}_r${rep}.err || exit $?
    timeout -k 10 120 python -u bench.py --graph $g --inflight 2 --cpu-sample 0 --no-e2e --steps 40 --warmup 10 \
      > $out/c2i2_g${g}_r${rep}.json 2> $out/c2i2_g${g}_r${rep}.err || exit $?
  done
done
