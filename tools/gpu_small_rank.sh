# per-rank shape of the 8-GPU strong-scaling run (1e8 / 8 = 1.25e7 rows) on one GPU: kernel vs superstep time
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/kmeans_kernel_bench.py --rows 12500000 --k 100 --iters 15 > gpurun_out/kmc_small.log 2>&1 && echo "kernel $(tail -1 gpurun_out/kmc_small.log)" || exit 1
timeout -k 10 300 python bench.py --rows 12500000 --steps 20 --warmup 3 --converge-iters 0 > gpurun_out/bench_small.log 2>&1 && echo "bench $(tail -1 gpurun_out/bench_small.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "ms/step")')" || exit 1
ALINK_TRACE=gpurun_out/small_trace_{rank}.json timeout -k 10 300 python bench.py --rows 12500000 --steps 10 --warmup 2 --converge-iters 0 > gpurun_out/small_trace.log 2>&1 || exit 1
python tools/trace_summary.py gpurun_out/small_trace_0.json > gpurun_out/small_trace_summary.txt
