#!/bin/bash
# round-5 GPU call: nearest counts mode (k-means|| weights in one pass) tests + convergence split + bench
set -o pipefail
LIMIT=400 TAG=km tools/gpu.sh tests tests/test_kmeans_kernel_gpu.py tests/test_kmeans_general_gpu.py || exit 1
tools/gpu.sh run initprof 300 python tools/kmeans_init_profile.py --reps 2 || exit 1
TAG=bench_y tools/gpu.sh bench || exit 1
