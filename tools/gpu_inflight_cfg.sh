#!/bin/bash
# bench.py --inflight 1 / 2 on configs 3 and 5 (alternating twice): does a second batch in flight fill their tails?
set -o pipefail
out=gpurun_out/inflight_cfg
mkdir -p $out
for rep in 1 2; do
  for k in 1 2; do
    timeout -k 10 120 python -u bench.py --inflight $k --horizon 20 --precision f32 --cpu-sample 0 --no-e2e --steps 30 \
      --warmup 5 > $out/c3_k${k}_r${rep}.json 2> $out/c3_k${k}_r${rep}.err || exit $?
    timeout -k 10 120 python -u bench.py --inflight $k --gait 1 --cpu-sample 0 --no-e2e --steps 30 --warmup 5 \
      > $out/c5_k${k}_r${rep}.json 2> $out/c5_k${k}_r${rep}.err || exit $?
  done
done
