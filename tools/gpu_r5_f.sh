#!/bin/bash
# round-5 GPU call: tree predict serving split + kernel profile
set -o pipefail
R=$PWD
tools/gpu.sh run treepred 400 python tools/tree_predict_bench.py --rows 2000000 --reps 1 || exit 1
tools/gpu.sh prof treepred 300 python $R/tools/tree_predict_bench.py --rows 500000 --reps 1 || exit 1
python tools/rocpd_stats.py gpurun_out/prof_treepred/treepred_results.db --top 15 > gpurun_out/prof_treepred_stats.txt 2>&1 || true
find gpurun_out -type f -size +1M ! -name '*.gz' -exec gzip -9 {} \;
