set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kmeans_kernel_gpu.py -q -x -k linear_grad --timeout 120 --timeout-method thread > gpurun_out/linear_tests.log 2>&1; rc=$?; tail -5 gpurun_out/linear_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python tools/linear_kernel_bench.py 20000000 > gpurun_out/linear_bench.json 2>&1 && cat gpurun_out/linear_bench.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_linear -o run -- python3 $GRAFT_REPO_ROOT/tools/linear_kernel_bench.py 20000000 32 > $GRAFT_REPO_ROOT/gpurun_out/prof_linear.log 2>&1 && echo PROF_OK
