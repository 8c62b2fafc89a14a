#!/bin/bash
# round 6: v10 time vs k (compute load per tile) at 1e8 rows, plus load-only / compute-only modes at k = 100
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
for k in 16 32 48 64 80 96 100 112; do
  tools/gpu.sh run kscan_$k 200 python tools/kmeans_kernel_bench.py --rows 100000000 --k $k --iters 15 --configs v10:1 --modes 0 || exit 1
done
tools/gpu.sh run kscan_modes 200 python tools/kmeans_kernel_bench.py --rows 100000000 --k 100 --iters 15 --configs v10:1 --modes 0,1,2,0,1,2 || exit 1
