#!/bin/bash
# round-4 GPU call F: fp32 quantize kernel tests + GBDT binning profile, then the full GPU suite
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
LIMIT=300 TAG=quant tools/gpu.sh tests tests/test_tree.py -k quantize || exit 1
tools/gpu.sh prof gbdt_q2 300 python $R/tools/gbdt_bench.py --rows 20000000 --features 1000 --trees 2 --depth 8 --dtype float32 --ranks 1 || exit 1
python tools/rocpd_stats.py gpurun_out/prof_gbdt_q2/gbdt_q2_results.db --top 8 > gpurun_out/prof_gbdt_q2_stats.txt 2>&1 || true
LIMIT=800 tools/gpu.sh tests tests/
rc=$?
find gpurun_out -type f -size +1M ! -name '*.gz' -exec gzip -9 {} \;
exit $rc
