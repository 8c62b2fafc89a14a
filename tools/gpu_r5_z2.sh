#!/bin/bash
# round-5 GPU call: first-cost kernel variants (rows in flight, load policy)
set -o pipefail
LIMIT=200 TAG=km tools/gpu.sh tests tests/test_kmeans_kernel_gpu.py -k "cost" || exit 1
COST1_ONLY=1 tools/gpu.sh run cost1 200 python tools/kmeans_nearest_bench.py || exit 1
