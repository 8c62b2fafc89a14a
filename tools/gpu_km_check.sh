# v7 (Plan<KB> ring) correctness + k=32/64/100/128 timings; one-shot all-reduce single-GPU tests
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kmeans_kernel_gpu.py tests/test_oneshot_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/kmc_tests.log 2>&1 && echo TESTS_OK || { tail -40 gpurun_out/kmc_tests.log; exit 1; }
tail -1 gpurun_out/kmc_tests.log
for k in 32 64 100 128; do
  for m in "" "--compute-only" "--load-only"; do
    timeout -k 10 200 python -u tools/kmeans_kernel_bench.py --k $k --iters 7 $m > gpurun_out/kmc.log 2>&1 || { echo "FAIL $k $m"; tail -20 gpurun_out/kmc.log; exit 1; }
    echo "k=$k $m $(tail -1 gpurun_out/kmc.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["hip_ms"],3), "ms", round(d["hip_rows_per_s"]/1e9,2), "e9 rows/s")')"
  done
done
