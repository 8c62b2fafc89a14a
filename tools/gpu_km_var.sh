# v7 tile scheduling A/B: VAR 1 (static chunks) vs VAR 3 (dynamic chunks from an atomic counter), at the 1-GPU
# headline shape (1e8 rows) and the 8-GPU per-rank shape (1.25e7 rows); correctness of both first
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 1 3; do
ALINK_KMEANS_V7_VAR=$v timeout -k 10 300 python -u -m pytest tests/test_kmeans_kernel_gpu.py -x -q -k "not linear and not search" --timeout 120 --timeout-method thread > gpurun_out/kmvar_tests.log 2>&1 && echo VAR${v}_TESTS_OK || { tail -40 gpurun_out/kmvar_tests.log; exit 1; }
done
for r in 1 2; do
for rows in 100000000 12500000; do
  for v in 1 3; do
    timeout -k 10 200 python -u tools/kmeans_kernel_bench.py --rows $rows --k 100 --iters 11 --var $v > gpurun_out/kmc.log 2>&1 || { echo "FAIL $rows $v"; tail -20 gpurun_out/kmc.log; exit 1; }
    echo "rows=$rows var=$v $(tail -1 gpurun_out/kmc.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["hip_ms"],3), "ms", round(d["hip_rows_per_s"]/1e9,2), "e9 rows/s")')"
  done
done
done
for v in 1 3; do
ALINK_KMEANS_V7_VAR=$v timeout -k 10 300 python bench.py --rows 12500000 --steps 20 --warmup 3 --converge-iters 0 > gpurun_out/bench_small.log 2>&1 && echo "bench rows=1.25e7 var=$v $(tail -1 gpurun_out/bench_small.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "ms/step")')" || exit 1
ALINK_KMEANS_V7_VAR=$v timeout -k 10 300 python bench.py --steps 20 --warmup 3 --converge-iters 0 > gpurun_out/bench_big.log 2>&1 && echo "bench rows=1e8 var=$v $(tail -1 gpurun_out/bench_big.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "ms/step")')" || exit 1
done
