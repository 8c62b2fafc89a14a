set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kmeans_kernel_gpu.py -x -q --timeout 120 --timeout-method thread -k "v7" > gpurun_out/pytest_v8.log 2>&1 && echo V8_TESTS_OK || { tail -40 gpurun_out/pytest_v8.log; exit 1; }
tail -1 gpurun_out/pytest_v8.log
for args in "--variant 8 --k 100" "--variant 8 --k 100 --load-only" "--variant 8 --k 100 --compute-only" "--variant 7 --k 100" "--variant 8 --k 32" "--variant 8 --k 64" "--variant 8 --k 128" "--variant 8 --k 112"; do
  timeout -k 10 120 python tools/kmeans_kernel_bench.py --rows 100000000 --iters 7 $args 2>/dev/null | tee -a gpurun_out/v8_diag.log || exit 1
done
