set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kmeans_kernel_gpu.py tests/test_e2e_gpu.py -q -x -m gpu -k "not linear and not search" --timeout 120 --timeout-method thread > gpurun_out/km_tests.log 2>&1 && echo KM_TESTS_OK || { tail -40 gpurun_out/km_tests.log; exit 1; }
tail -1 gpurun_out/km_tests.log
for r in 1 2; do
timeout -k 10 200 python -u tools/kmeans_kernel_bench.py --k 100 --iters 9 > gpurun_out/kmc.log 2>&1 && echo "kernel k=100 $(tail -1 gpurun_out/kmc.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["hip_ms"],3), "ms")')" || exit 1
timeout -k 10 500 python bench.py --steps 20 --warmup 3 --converge-iters 0 > gpurun_out/bench.log 2>&1 && echo "bench $(tail -1 gpurun_out/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "ms/step", round(d["value"]/1e9,2), "e9 rows/s")')" || exit 1
done
timeout -k 10 500 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log > gpurun_out/bench.json && cat gpurun_out/bench.json || exit 1
ALINK_TRACE=gpurun_out/bench_trace_{rank}.json timeout -k 10 300 python bench.py --steps 10 --warmup 2 --converge-iters 0 > gpurun_out/bench_trace.log 2>&1 || { tail -20 gpurun_out/bench_trace.log; exit 1; }
python tools/trace_summary.py gpurun_out/bench_trace_0.json | tee gpurun_out/bench_trace_summary.txt
