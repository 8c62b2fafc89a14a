# v7 vs v7-PF (distance fragments of tile i+1 read after barrier i): correctness + k=64/100/128 timings, alternated
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
ALINK_KMEANS_V7_PF=1 timeout -k 10 300 python -u -m pytest tests/test_kmeans_kernel_gpu.py -x -q -k "not linear" --timeout 120 --timeout-method thread > gpurun_out/kmpf_tests.log 2>&1 && echo PF_TESTS_OK || { tail -40 gpurun_out/kmpf_tests.log; exit 1; }
for k in 100 128 64 100; do
  for m in "" "--pf" "--compute-only" "--compute-only --pf"; do
    timeout -k 10 200 python -u tools/kmeans_kernel_bench.py --k $k --iters 9 $m > gpurun_out/kmc.log 2>&1 || { echo "FAIL $k $m"; tail -20 gpurun_out/kmc.log; exit 1; }
    echo "k=$k $m $(tail -1 gpurun_out/kmc.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["hip_ms"],3), "ms", round(d["hip_rows_per_s"]/1e9,2), "e9 rows/s")')"
  done
done
