# v7 VAR 1 (default) vs VAR 4 (VAR 1 + tree argmax), interleaved 3 rounds, full and compute-only
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
ALINK_KMEANS_V7_VAR=4 timeout -k 10 300 python -u -m pytest tests/test_kmeans_kernel_gpu.py -x -q -k "not linear and not search" --timeout 120 --timeout-method thread > gpurun_out/kmvar_tests.log 2>&1 && echo VAR4_TESTS_OK || { tail -40 gpurun_out/kmvar_tests.log; exit 1; }
for r in 1 2 3; do
for k in 100 128; do
  for m in "--var 1" "--var 4" "--compute-only --var 1" "--compute-only --var 4"; do
    timeout -k 10 200 python -u tools/kmeans_kernel_bench.py --k $k --iters 9 $m > gpurun_out/kmc.log 2>&1 || { echo "FAIL $k $m"; tail -20 gpurun_out/kmc.log; exit 1; }
    echo "k=$k $m $(tail -1 gpurun_out/kmc.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["hip_ms"],3), "ms", round(d["hip_rows_per_s"]/1e9,2), "e9 rows/s")')"
  done
done
done
