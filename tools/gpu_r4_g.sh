#!/bin/bash
# round-4 GPU call G (E + F in one box): new-kernel tests, KMeans v10 A/B, FTRL pipeline with the CSR SpMV,
# transfer-site count, GBDT binning profile, PMC passes, full GPU suite
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
LIMIT=300 TAG=newk tools/gpu.sh tests tests/test_feature_gpu.py tests/test_tree.py -k "csr_mv or quantize" || exit 1
tools/gpu.sh run kmeans_ab2 400 python tools/kmeans_ab.py --rounds 4 --libs base=alink_amd/ops/libalink_hip.so,dot2=variants/libalink_hip_dot2.so,dot2pair=variants/libalink_hip_dot2pair.so --modes 0 --iters 20 || exit 1
tools/gpu.sh run ftrl_pipe_sharded_32m_csrmv 240 python tools/ftrl_pipeline_bench.py --mode SHARDED --rows 32000000 || exit 1
tools/gpu.sh run ftrl_sync 240 python tools/ftrl_sync_count.py --rows 2097152 || exit 1
tools/gpu.sh prof gbdt_q2 300 python $R/tools/gbdt_bench.py --rows 20000000 --features 1000 --trees 2 --depth 8 --dtype float32 --ranks 1 || exit 1
python tools/rocpd_stats.py gpurun_out/prof_gbdt_q2/gbdt_q2_results.db --top 8 > gpurun_out/prof_gbdt_q2_stats.txt 2>&1 || true
VARIANT=dot2pair tools/gpu_r4_c.sh || exit 1
LIMIT=700 tools/gpu.sh tests tests/
rc=$?
find gpurun_out -type f -size +1M ! -name '*.gz' -exec gzip -9 {} \;
exit $rc
