#!/bin/bash
# round-5 GPU call: GBDT per-tree timeline (gaps between kernels) at the per-rank config-3 shape
set -o pipefail
R=$PWD
tools/gpu.sh prof gbdt 600 python $R/tools/gbdt_bench.py --rows 12500000 --features 1000 --trees 6 --depth 8 --dtype float32 || exit 1
python tools/rocpd_stats.py gpurun_out/prof_gbdt/gbdt_results.db --top 30 --timeline "tree_hist_fm<3, false" --steady 5 > gpurun_out/prof_gbdt_stats.txt 2>&1 || true
find gpurun_out -type f -size +1M ! -name '*.gz' -exec gzip -9 {} \;
