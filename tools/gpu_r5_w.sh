#!/bin/bash
# round-5 GPU call: nearest-kernel RG A/B (+ tests), then the 8-process one-GPU KMeans rehearsal
set -o pipefail
R=$PWD
LIMIT=300 TAG=near tools/gpu.sh tests tests/test_kmeans_kernel_gpu.py -k nearest || exit 1
tools/gpu.sh run nearest 300 python tools/kmeans_nearest_bench.py || exit 1
tools/gpu_r5_v.sh
