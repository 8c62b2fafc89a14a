#!/bin/bash
# round-5 GPU call: kernel timeline of the 8-GPU per-rank shape (1.25e7 rows) bench step
set -o pipefail
R=$PWD
tools/gpu.sh prof k125 300 python $R/bench.py --rows 12500000 --steps 50 --warmup 5 --converge-iters 0 || exit 1
python tools/rocpd_stats.py gpurun_out/prof_k125/k125_results.db --top 12 --timeline kmeans_v10 > gpurun_out/prof_k125_stats.txt 2>&1 || true
find gpurun_out -type f -size +1M ! -name '*.gz' -exec gzip -9 {} \;
