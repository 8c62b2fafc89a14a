#!/bin/bash
# KMeans: kernel numerics tests, kernel trace of the 1-GPU bench (per-step kernel sequence + gaps), bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_kmeans_kernel_gpu.py tests/test_kmeans.py -x -q > gpurun_out/kmprof_tests.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kmprof -o run -- \
  python3 bench.py --steps 10 --warmup 2 --converge-iters 0 > gpurun_out/kmprof.log 2>&1 &&
timeout -k 10 600 python bench.py > gpurun_out/km_bench.log 2>&1
rc=$?
tail -2 gpurun_out/kmprof_tests.log; tail -1 gpurun_out/km_bench.log | cut -c1-400
exit $rc
