#!/bin/bash
# round-5 GPU call: KMeans convergence word (skipped speculative launch) tests + convergence-run split + bench
set -o pipefail
LIMIT=400 TAG=km tools/gpu.sh tests tests/test_kmeans_kernel_gpu.py tests/test_kmeans_general_gpu.py tests/test_multiprocess_gpu.py -k "kmeans or KMeans" || exit 1
tools/gpu.sh run initprof 300 python tools/kmeans_init_profile.py --reps 2 || exit 1
TAG=bench_x tools/gpu.sh bench || exit 1
