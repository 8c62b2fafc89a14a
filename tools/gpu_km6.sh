#!/bin/bash
# v6 KMeans kernel: numerics tests, variant timing at k=100 (full / compute-only), 1-GPU bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_kmeans_kernel_gpu.py -x -q -m gpu > gpurun_out/km6_tests.log 2>&1 &&
timeout -k 10 300 python tools/kmeans_kernel_bench.py --variant 6 --k 100 > gpurun_out/km6_k100.log 2>&1 &&
timeout -k 10 300 python tools/kmeans_kernel_bench.py --variant 6 --k 100 --compute-only > gpurun_out/km6_k100_compute.log 2>&1 &&
timeout -k 10 300 python tools/kmeans_kernel_bench.py --variant 6 --k 128 > gpurun_out/km6_k128.log 2>&1 &&
timeout -k 10 600 python bench.py > gpurun_out/km6_bench.log 2>&1
rc=$?
tail -3 gpurun_out/km6_tests.log; cat gpurun_out/km6_k100*.log gpurun_out/km6_k128.log | grep -v "^$" | tail -12; tail -2 gpurun_out/km6_bench.log
exit $rc
