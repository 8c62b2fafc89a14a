#!/bin/bash
# A/B of v6 KMeans kernel builds: in-tree lib vs build/exp/lib*.so (numerics test on each), k=100
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python tools/kmeans_kernel_bench.py --variant 6 --k 100 > gpurun_out/ab_default.log 2>&1 || exit 1
for lib in build/exp/lib*.so; do
  n=$(basename $lib .so)
  ALINK_HIP_LIB=$lib timeout -k 10 600 python -m pytest tests/test_kmeans_kernel_gpu.py -x -q > gpurun_out/ab_tests_$n.log 2>&1 || exit 1
  ALINK_HIP_LIB=$lib timeout -k 10 300 python tools/kmeans_kernel_bench.py --variant 6 --k 100 > gpurun_out/ab_$n.log 2>&1 || exit 1
done
for f in gpurun_out/ab_tests_*.log; do echo "$f $(tail -1 $f)"; done
for f in gpurun_out/ab_default.log gpurun_out/ab_lib*.log; do echo "$f $(grep -o '"hip_ms": [0-9.]*' $f)"; done
