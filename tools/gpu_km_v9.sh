# v9 vs v7: kernel tests under both, then the k=100 bench of each (full / load-only / compute-only)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
ALINK_KMEANS_KERNEL=v9 timeout -k 10 300 python -u -m pytest tests/test_kmeans_kernel_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/v9_tests.log 2>&1 && echo V9_TESTS_OK || { tail -40 gpurun_out/v9_tests.log; exit 1; }
for v in v7 v9; do
  for m in "" "--compute-only" "--load-only"; do
    ALINK_KMEANS_KERNEL=$v timeout -k 10 200 python -u tools/kmeans_kernel_bench.py --k 100 --iters 7 $m > gpurun_out/km_$v.log 2>&1 || { echo "FAIL $v $m"; tail -20 gpurun_out/km_$v.log; exit 1; }
    echo "$v $m $(tail -1 gpurun_out/km_$v.log)"
  done
done
