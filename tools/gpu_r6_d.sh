#!/bin/bash
# round 6: v10 L2 prefetch distance A/B (ALINK_KMEANS_V10_PFD), 1e8 and 1.25e7 rows
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
LIMIT=200 tools/gpu.sh tests tests/test_kmeans_kernel_gpu.py -k "prefetch" || exit 1
tools/gpu.sh run pfd_ab 400 python tools/kmeans_kernel_bench.py --rows 100000000 --k 100 --iters 20 --sub-rows 12500000 --configs v10:1,v10:1f2,v10:1f4,v10:1f8,v10:1f12,v10:1,v10:1f4,v10:1f8 --modes 0 || exit 1
