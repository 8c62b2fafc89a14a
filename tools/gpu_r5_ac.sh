#!/bin/bash
# round-5 GPU call: host-side compaction in the fused KMeans update (no first-use torch kernels in the supersteps)
set -o pipefail
LIMIT=400 TAG=km tools/gpu.sh tests tests/test_kmeans_kernel_gpu.py tests/test_kmeans_general_gpu.py tests/test_multiprocess_gpu.py -k "kmeans or KMeans" || exit 1
tools/gpu.sh run firstrun 300 python tools/kmeans_first_run_trace.py || exit 1
TAG=bench_w3 tools/gpu.sh bench --steps 20 --warmup 3 || exit 1
TAG=bench_w5 tools/gpu.sh bench --steps 20 --warmup 5 --converge-iters 0 || exit 1
