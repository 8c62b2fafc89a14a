#!/bin/bash
# round-5 GPU call: GBDT level host work (batched sibling subtraction, vectorised split materialisation, uint8
# slot sort): tree GPU tests, bench, per-tree timeline
set -o pipefail
R=$PWD
LIMIT=500 tools/gpu.sh tests tests/test_tree.py tests/test_tree_predict_gpu.py tests/test_gbdt_rank_gpu.py tests/test_multiprocess_gpu.py || exit 1
tools/gpu.sh run gbdt 600 python tools/gbdt_bench.py --rows 12500000 --features 1000 --trees 20 --depth 8 --dtype float32 || exit 1
tools/gpu.sh prof gbdt 600 python $R/tools/gbdt_bench.py --rows 12500000 --features 1000 --trees 6 --depth 8 --dtype float32 || exit 1
python tools/rocpd_stats.py gpurun_out/prof_gbdt/gbdt_results.db --top 30 --timeline "tree_hist_fm<3, false" --steady 5 > gpurun_out/prof_gbdt_stats.txt 2>&1 || true
find gpurun_out -type f -size +1M ! -name '*.gz' -exec gzip -9 {} \;
