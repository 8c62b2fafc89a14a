# top-K kernel: GPU tests + throughput bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_topk_gpu.py tests/test_als.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/topk_tests.log 2>&1 && echo TESTS_OK || { tail -40 gpurun_out/topk_tests.log; exit 1; }
timeout -k 10 300 python -u tools/topk_bench.py > gpurun_out/topk_bench.log 2>&1 && echo BENCH_OK || { tail -30 gpurun_out/topk_bench.log; exit 1; }
cat gpurun_out/topk_bench.log
