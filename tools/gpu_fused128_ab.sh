#!/bin/bash
# A/B of the fp64 128 class fused (k_solve128<double>: condensing + IPM in one launch, --path FUSED128=1) against the
# default two launches, on the headline (empty 128 class) and config 5 (1309 QPs of n = 120), alternating twice.
set -o pipefail
out=gpurun_out/f128
mkdir -p $out
for rep in 1 2; do
  for f in 0 1; do
    timeout -k 10 120 python -u bench.py --path FUSED128=$f --cpu-sample 0 --no-e2e --steps 60 --warmup 10 \
      > $out/c2_f${f}_r${rep}.json 2> $out/c2_f${f}_r${rep}.err || exit $?
    timeout -k 10 120 python -u bench.py --path FUSED128=$f --gait 1 --cpu-sample 0 --no-e2e --steps 40 --warmup 10 \
      > $out/c5_f${f}_r${rep}.json 2> $out/c5_f${f}_r${rep}.err || exit $?
  done
done
