#!/bin/bash
# Session script (round 5): finer chain stamps; bench --ocp projected / rows at B=1 (tick line, single-thread CPU);
# the headline bench with --cadence 20
O=gpurun_out/r05i; mkdir -p $O
CMPC_LIB=lab/_stamps/libcmpc_ocpstamps.so timeout -k 10 200 python -u tools/ocp_probe.py --stamps > $O/stamps.log 2>&1 || { cat $O/stamps.log; exit 8; }
timeout -k 10 300 python -u bench.py --ocp projected --batch 1 --steps 200 --warmup 20 > $O/bench_ocp_projected_b1.json 2> $O/bench_ocp_p.err || { tail -20 $O/bench_ocp_p.err; exit 7; }
timeout -k 10 300 python -u bench.py --ocp rows --batch 1 --steps 50 --warmup 5 > $O/bench_ocp_rows_b1.json 2> $O/bench_ocp_r.err || { tail -20 $O/bench_ocp_r.err; exit 6; }
timeout -k 10 300 python -u bench.py --cadence 20 > $O/bench_cadence.json 2> $O/bench_cad.err || { tail -20 $O/bench_cad.err; exit 5; }
echo done
