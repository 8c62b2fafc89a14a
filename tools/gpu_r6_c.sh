#!/bin/bash
# round 6: nearest kernel RG 3/4 A/B (k-means|| weights pass)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
LIMIT=200 tools/gpu.sh tests tests/test_kmeans_kernel_gpu.py -k "two_row_groups or counts" || exit 1
RG_AB=1 tools/gpu.sh run rg_ab 300 python tools/kmeans_nearest_bench.py --reps 5 || exit 1
