#!/bin/bash
# round-5 GPU call: tree tests, RF per-level host time after the batched shuffles / transfers / parking
set -o pipefail
LIMIT=400 tools/gpu.sh tests tests/test_tree.py tests/test_tree_predict_gpu.py tests/test_gbdt_rank_gpu.py || exit 1
tools/gpu.sh run rflevels 600 python tools/rf_level_bench.py --rows 1000000 --features 100 || exit 1
tools/gpu.sh run rf_cprof 600 python -m cProfile -o gpurun_out/rf.prof tools/rf_level_bench.py --rows 1000000 --features 100 || exit 1
