#!/bin/bash
# round-5 GPU call: sync-free FTRL shard update + one-launch FeatureHasher; RF parked levels
set -o pipefail
R=$PWD
LIMIT=500 tools/gpu.sh tests tests/test_ftrl_gpu.py tests/test_strings_gpu.py tests/test_feature_gpu.py tests/test_tree_predict_gpu.py || exit 1
tools/gpu.sh run ftrl32 300 python tools/ftrl_pipeline_bench.py --rows 32000000 || exit 1
tools/gpu.sh run rflevels 600 python tools/rf_level_bench.py --rows 1000000 --features 100 || exit 1
tools/gpu.sh run gbdt_cprof 600 python -m cProfile -o gpurun_out/gbdt.prof tools/gbdt_bench.py --rows 12500000 --features 1000 --trees 6 --depth 8 --dtype float32 || exit 1
