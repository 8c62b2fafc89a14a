#!/bin/bash
# round-4 GPU call H: the dot2 accumulate as production default -- KMeans GPU tests, A/B against the former
# d16 layout, PMC of both, the headline bench; FTRL pipeline after the eval / hasher host-side cuts
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LIMIT=400 TAG=km tools/gpu.sh tests tests/test_kmeans.py tests/test_kmeans_fp32_gpu.py tests/test_kmeans_general_gpu.py tests/test_kmeans_kernel_gpu.py tests/test_kmeans_operand_hysteresis.py || exit 1
tools/gpu.sh run kmeans_ab3 400 python tools/kmeans_ab.py --rounds 4 --libs dot2=alink_amd/ops/libalink_hip.so,d16=variants/libalink_hip_d16.so --modes 0 --iters 20 || exit 1
LIMIT=300 tools/gpu.sh bench || exit 1
VARIANT=d16 tools/gpu_r4_c.sh || exit 1
tools/gpu.sh run ftrl_pipe_sharded_32m_h 240 python tools/ftrl_pipeline_bench.py --mode SHARDED --rows 32000000 || exit 1
tools/gpu.sh run ftrl_sync_h 240 python tools/ftrl_sync_count.py --rows 2097152 || exit 1
find gpurun_out -type f -size +1M ! -name '*.gz' -exec gzip -9 {} \;
