#!/bin/bash
# Session script: OCP B = 1 latency A/B on one box — HEAD vs dc12ddd (MFMA T) vs f8870e7 (two pivots per barrier).
O=gpurun_out/r04n; mkdir -p $O
export OCP_REPS=30
for i in 1 2; do
  for L in head:cheeta-mpc_amd/lib/libcmpc.so dc12:lab/_ab/libcmpc_dc12.so f887:lab/_ab/libcmpc_f887.so; do
    n=${L%%:*}; CMPC_LIB=${L#*:} timeout -k 10 200 python -u tools/ocp_probe.py 1 256 > $O/$n$i.log 2>&1 || { cat $O/$n$i.log; exit 9; }
    sed "s/^/$n$i /" $O/$n$i.log
  done
done
