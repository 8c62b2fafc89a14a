set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kmeans_kernel_gpu.py tests/test_trace_metrics.py tests/test_linear_gpu.py -q -x -m gpu -k "linear or trace or sparse or hashed" --timeout 120 --timeout-method thread > gpurun_out/linear_tests.log 2>&1; rc=$?; tail -3 gpurun_out/linear_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python tools/linear_kernel_bench.py 20000000 > gpurun_out/linear_bench.json 2>&1 && cat gpurun_out/linear_bench.json
