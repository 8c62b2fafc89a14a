#!/bin/bash
# round-6 regression check: the v10 kernel from the round-5 library vs HEAD, interleaved, one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for lib in variants/libalink_hip_r5.so alink_amd/ops/libalink_hip.so; do
    echo "== round $r lib $lib"
    ALINK_HIP_LIB=$PWD/$lib timeout -k 10 120 python -u tools/kmeans_kernel_bench.py --rows 100000000 --k 100 \
      --iters 20 --configs v10:2 --modes 0 --sub-rows 12500000 || exit 1
  done
done
