#!/bin/bash
# round-5 GPU call: KMeans kernel tests + init phase profile
set -o pipefail
LIMIT=200 tools/gpu.sh tests tests/test_kmeans_kernel_gpu.py || exit 1
tools/gpu.sh run initprof 300 python tools/kmeans_init_profile.py --rows 100000000 --reps 3 || exit 1
