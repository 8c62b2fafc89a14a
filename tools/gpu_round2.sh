set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/variants.log
timeout -k 10 300 python -m pytest tests/test_kmeans_kernel_gpu.py -x -q > gpurun_out/kt.log 2>&1 && echo PYTEST_OK || { tail -30 gpurun_out/kt.log; exit 1; }
for k in 100 64 128 32; do for v in 1 4 5; do timeout -k 10 200 python tools/kmeans_kernel_bench.py --rows 100000000 --k $k --iters 7 --variant $v >> gpurun_out/variants.log 2>&1 || exit 1; done; done
grep rows gpurun_out/variants.log
timeout -k 10 400 python bench.py --steps 20 --warmup 3 > gpurun_out/bench2.log 2>&1 && echo BENCH_OK && tail -1 gpurun_out/bench2.log
