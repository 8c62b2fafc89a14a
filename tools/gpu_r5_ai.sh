#!/bin/bash
# round-5 GPU call: update-stat wait by host poll of a sequence word vs stream event (A/B at the per-rank shape)
set -o pipefail
R=$PWD
ALINK_KMEANS_HOST_POLL=1 LIMIT=300 TAG=kmpoll tools/gpu.sh tests tests/test_kmeans_kernel_gpu.py -k "speculative or compaction or skip or update" || exit 1
for v in 0 1 0 1; do
  ALINK_KMEANS_HOST_POLL=$v TAG=poll$v tools/gpu.sh bench --rows 12500000 --steps 100 --warmup 40 --converge-iters 0 || exit 1
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/poll$v.json
done
for v in 0 1; do
  ALINK_KMEANS_HOST_POLL=$v tools/gpu.sh prof p$v 300 python $R/bench.py --rows 12500000 --steps 60 --warmup 40 --converge-iters 0 || exit 1
  python tools/rocpd_stats.py gpurun_out/prof_p$v/p${v}_results.db --top 3 --timeline kmeans_v10 --steady 50 > gpurun_out/prof_p${v}_stats.txt 2>&1 || true
  tail -7 gpurun_out/prof_p${v}_stats.txt
done
find gpurun_out -type f -size +1M ! -name '*.gz' -exec gzip -9 {} \;
