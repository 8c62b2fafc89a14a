#!/bin/bash
# round-4 GPU call A: full GPU suite, v10 variant correctness, v10 variant A/B timing (one box)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LIMIT=700 tools/gpu.sh tests tests/ || exit 1
for v in pk pair pkpair dot2 dot2pair; do
  TAG=var_$v LIMIT=200 ALINK_HIP_LIB=$PWD/variants/libalink_hip_$v.so tools/gpu.sh tests tests/test_kmeans_kernel_gpu.py || exit 1
done
tools/gpu.sh run kmeans_ab 500 python tools/kmeans_ab.py --rounds 2 --libs base=alink_amd/ops/libalink_hip.so,pk=variants/libalink_hip_pk.so,pair=variants/libalink_hip_pair.so,pkpair=variants/libalink_hip_pkpair.so,dot2=variants/libalink_hip_dot2.so,dot2pair=variants/libalink_hip_dot2pair.so --modes 0,2 --sub-rows 12500000
