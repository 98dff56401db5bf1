R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -2 gpurun_out/gpu_tests.log; [ $rc -ne 0 ] && exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py --steps 10 --cpu-sample 0 > $R/gpurun_out/prof.log 2>&1 || exit 1
grep -E 'class_lists|ipm64' $R/gpurun_out/prof/run_kernel_stats.csv | cut -d, -f1-4
