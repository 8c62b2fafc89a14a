#!/bin/bash
# round-5 GPU call: headline KMeans step A/B (serpentine on/off, interleaved) + kernel-trace profile of bench.py
set -o pipefail
R=$PWD
for i in 1 2; do
  TAG=b_s1_$i tools/gpu.sh bench --steps 20 --warmup 3 --converge-iters 0 || exit 1
  ALINK_KMEANS_SERPENTINE=0 TAG=b_s0_$i tools/gpu.sh bench --steps 20 --warmup 3 --converge-iters 0 || exit 1
done
TAG=b125_s1 tools/gpu.sh bench --rows 12500000 --steps 50 --warmup 5 --converge-iters 0 || exit 1
ALINK_KMEANS_SERPENTINE=0 TAG=b125_s0 tools/gpu.sh bench --rows 12500000 --steps 50 --warmup 5 --converge-iters 0 || exit 1
tools/gpu.sh prof kbench 300 python $R/bench.py --steps 20 --warmup 3 --converge-iters 0 || exit 1
python tools/rocpd_stats.py gpurun_out/prof_kbench/kbench_results.db --top 15 --timeline kmeans_v10 > gpurun_out/prof_kbench_stats.txt 2>&1 || true
find gpurun_out -type f -size +1M ! -name '*.gz' -exec gzip -9 {} \;
