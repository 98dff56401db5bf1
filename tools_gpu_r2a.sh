#!/bin/bash
# GPU-box script (round 2): GPU tests, headline bench, config-4 full batch bench, 2-rank gather rehearsal on one GPU.
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit 1;; esac; }
(lscpu | head -20; nproc; cat /sys/fs/cgroup/cpu.max 2>/dev/null; echo OMP=$OMP_NUM_THREADS) > $O/host_cpu.txt 2>&1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -6 $O/gpu_tests.log; echo tests_rc=$rc; fatal $rc tests; [ $rc -ne 0 ] && exit 1
timeout -k 10 200 python bench.py > $O/bench_head.json 2> $O/bench_head.err; rc=$?; echo bench_rc=$rc; cat $O/bench_head.json; fatal $rc bench
timeout -k 10 200 python bench.py --batch 262144 --steps 5 --cpu-sample 0 > $O/bench_c4.json 2> $O/bench_c4.err; rc=$?; echo c4_rc=$rc; cat $O/bench_c4.json; fatal $rc c4
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --cpu-sample 0 > $O/bench_2r.json 2> $O/bench_2r.err; rc=$?; echo 2r_rc=$rc; cat $O/bench_2r.json; fatal $rc 2r
echo all_done
