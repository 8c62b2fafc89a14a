#!/bin/bash
# round-4 GPU call I: where the headline step's time goes outside the fused kernel (full and per-rank 8-GPU
# shape), kernel-trace only
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
tools/gpu.sh prof bench_full 300 python $R/bench.py --steps 10 --warmup 3 --converge-iters 0 || exit 1
python tools/rocpd_stats.py gpurun_out/prof_bench_full/bench_full_results.db --top 12 --timeline kmeans_v10 > gpurun_out/prof_bench_full_stats.txt 2>&1 || true
tools/gpu.sh prof bench_rank8 300 python $R/bench.py --rows 12500000 --steps 20 --warmup 3 --converge-iters 0 || exit 1
python tools/rocpd_stats.py gpurun_out/prof_bench_rank8/bench_rank8_results.db --top 12 --timeline kmeans_v10 > gpurun_out/prof_bench_rank8_stats.txt 2>&1 || true
LIMIT=200 tools/gpu.sh bench --rows 12500000 --steps 50 --warmup 5 --converge-iters 0 || exit 1
find gpurun_out -type f -size +1M ! -name '*.gz' -exec gzip -9 {} \;
