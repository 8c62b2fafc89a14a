set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kmeans_kernel_gpu.py -x -q -k nearest --timeout 120 --timeout-method thread > gpurun_out/nearest.log 2>&1; rc=$?; tail -15 gpurun_out/nearest.log; [ $rc = 0 ] || exit $rc
timeout -k 10 500 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log
