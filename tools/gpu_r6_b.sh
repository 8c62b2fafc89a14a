#!/bin/bash
# round 6: tree code kernel occupancy fix; GBDT config 3 full-size kernel split
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
LIMIT=300 tools/gpu.sh tests tests/test_tree_predict_gpu.py || exit 1
tools/gpu.sh run treebench_v3 400 python tools/tree_predict_bench.py --reps 3 || exit 1
tools/gpu.sh prof treepred3 300 python "$R/tools/tree_predict_bench.py" --rows 500000 --reps 1 || exit 1
tools/gpu.sh prof gbdtfull 600 python "$R/tools/gbdt_bench.py" --rows 100000000 --features 1000 --trees 3 --depth 8 --prebinned 1 || exit 1
tools/gpu.sh pmc gbdtfull "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" 300 python "$R/tools/gbdt_bench.py" --rows 100000000 --features 1000 --trees 1 --depth 8 --prebinned 1 || exit 1
LIMIT=200 tools/gpu.sh tests tests/test_kmeans_kernel_gpu.py -k "counts or seed_ref" || exit 1
COUNTS_AB=1 tools/gpu.sh run counts_ab 200 python tools/kmeans_nearest_bench.py --reps 5 || exit 1
ALINK_TELEMETRY_OUT=gpurun_out/tel_c.json TAG=bench_c tools/gpu.sh bench || exit 1
