#!/bin/bash
# round-5 GPU call: nearest kernel with two centroid blocks per step (A/B, identity tests)
set -o pipefail
LIMIT=300 TAG=km tools/gpu.sh tests tests/test_kmeans_kernel_gpu.py -k "nearest or cost" || exit 1
BP_AB=1 tools/gpu.sh run bp 200 python tools/kmeans_nearest_bench.py || exit 1
