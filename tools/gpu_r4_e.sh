#!/bin/bash
# round-4 GPU call E: CSR SpMV kernel test, FTRL pipeline with it (+ transfer-site count), longer KMeans A/B of
# the two dot2 variants against production, PMC passes (production vs dot2pair)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LIMIT=200 TAG=csrmv tools/gpu.sh tests tests/test_feature_gpu.py || exit 1
tools/gpu.sh run ftrl_pipe_sharded_32m_csrmv 240 python tools/ftrl_pipeline_bench.py --mode SHARDED --rows 32000000 || exit 1
tools/gpu.sh run ftrl_sync 240 python tools/ftrl_sync_count.py --rows 2097152 || exit 1
tools/gpu.sh run kmeans_ab2 500 python tools/kmeans_ab.py --rounds 4 --libs base=alink_amd/ops/libalink_hip.so,dot2=variants/libalink_hip_dot2.so,dot2pair=variants/libalink_hip_dot2pair.so --modes 0 --iters 20 || exit 1
VARIANT=dot2pair tools/gpu_r4_c.sh
rc=$?
find gpurun_out -type f -size +1M ! -name '*.gz' -exec gzip -9 {} \;
exit $rc
