#!/bin/bash
# round 6: tree serving A/B + profile, GBDT config 3 at full size (prebinned), one MI355X
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
LIMIT=300 tools/gpu.sh tests tests/test_tree_predict_gpu.py || exit 1
ALINK_TREE_PREDICT_KERNEL=1 tools/gpu.sh run treebench_v1 400 python tools/tree_predict_bench.py --reps 3 || exit 1
tools/gpu.sh run treebench_v2 400 python tools/tree_predict_bench.py --reps 3 || exit 1
tools/gpu.sh run treebench_v2_miss 400 python tools/tree_predict_bench.py --reps 3 --rows 1000000 --missing 0.05 || exit 1
tools/gpu.sh prof treepred 300 python "$R/tools/tree_predict_bench.py" --rows 500000 --reps 1 || exit 1
tools/gpu.sh pmc treepred "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE" 120 python "$R/tools/tree_predict_bench.py" --rows 500000 --reps 1 || exit 1
tools/gpu.sh run gbdt_full 900 python tools/gbdt_bench.py --rows 100000000 --features 1000 --trees 20 --depth 8 --prebinned 1 || exit 1
