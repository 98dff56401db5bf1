R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; echo tests_rc=$rc; [ $rc -ne 0 ] && exit 1
timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 10 --warmup 2 > gpurun_out/bench2.json 2> gpurun_out/bench2.err; rc=$?; echo bench2_rc=$rc; cat gpurun_out/bench2.json; tail -3 gpurun_out/bench2.err
