#!/bin/bash
# round-5 GPU call: packed GBDT histogram (K7) — tests, per-rank config-3 shape A/B, PMC before/after
set -o pipefail
R=$PWD
LIMIT=400 tools/gpu.sh tests tests/test_tree.py || exit 1
ALINK_TREE_HIST_PACK=0 tools/gpu.sh run gbdt_plain 500 python tools/gbdt_bench.py --rows 12500000 --features 1000 --trees 20 --depth 8 --dtype float32 || exit 1
tools/gpu.sh run gbdt_pack 500 python tools/gbdt_bench.py --rows 12500000 --features 1000 --trees 20 --depth 8 --dtype float32 || exit 1
tools/gpu.sh pmc hist_pack "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT" 240 python $R/tools/gbdt_bench.py --rows 2000000 --features 1000 --trees 2 --depth 8 --dtype float32 || exit 1
tools/gpu.sh prof gbdt_pack 300 python $R/tools/gbdt_bench.py --rows 12500000 --features 1000 --trees 4 --depth 8 --dtype float32 || exit 1
python tools/rocpd_stats.py gpurun_out/prof_gbdt_pack/gbdt_pack_results.db --top 14 > gpurun_out/prof_gbdt_pack_stats.txt 2>&1 || true
find gpurun_out -type f -size +1M ! -name '*.gz' -exec gzip -9 {} \;
