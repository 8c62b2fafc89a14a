#!/bin/bash
# round-5 GPU call: counts-mode argmax A/B (exact vs packed-index max), nearest tests
set -o pipefail
LIMIT=300 TAG=km tools/gpu.sh tests tests/test_kmeans_kernel_gpu.py -k "nearest or cost" || exit 1
PACKED_AB=1 tools/gpu.sh run packed 200 python tools/kmeans_nearest_bench.py || exit 1
