#!/bin/bash
# round-5 GPU call: tree predict kernel tests + serving throughput
set -o pipefail
LIMIT=400 tools/gpu.sh tests tests/test_tree_predict_gpu.py tests/test_tree.py || exit 1
tools/gpu.sh run treepred 400 python tools/tree_predict_bench.py --rows 2000000 --trees 500 --depth 8 --features 1000 || exit 1
tools/gpu.sh run treepred_miss 300 python tools/tree_predict_bench.py --rows 1000000 --trees 500 --depth 8 --features 1000 --missing 0.05 --reps 2 || exit 1
