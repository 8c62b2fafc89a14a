set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/ -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK
timeout -k 10 400 python bench.py --steps 20 --warmup 3 > gpurun_out/bench1.log 2>&1 && echo BENCH_OK
for v in 1 2; do timeout -k 10 200 python tools/kmeans_kernel_bench.py --rows 100000000 --k 64 --iters 5 --variant $v >> gpurun_out/variants.log 2>&1; done
tail -3 gpurun_out/pytest_gpu.log; tail -2 gpurun_out/smoke.log; tail -2 gpurun_out/bench1.log; cat gpurun_out/variants.log | grep rows
