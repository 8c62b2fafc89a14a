#!/bin/bash
# round-5 GPU call: streaming first-cost kernel (tests, A/B vs the nearest m=1 pass) + convergence split + bench
set -o pipefail
LIMIT=400 TAG=km tools/gpu.sh tests tests/test_kmeans_kernel_gpu.py tests/test_kmeans_general_gpu.py || exit 1
COST1_ONLY=1 tools/gpu.sh run cost1 200 python tools/kmeans_nearest_bench.py || exit 1
tools/gpu.sh run initprof 300 python tools/kmeans_init_profile.py --reps 2 || exit 1
TAG=bench_z tools/gpu.sh bench || exit 1
