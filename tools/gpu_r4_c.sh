#!/bin/bash
# round-4 GPU call C: PMC counters of the fused KMeans v10 kernel, production build vs one variant build
# (VARIANT=pk|pair|pkpair|dot2|dot2pair), two passes each (instruction mix; busy / stall cycles).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
V=${VARIANT:-pkpair}
P1="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA"
B="python $PWD/tools/kmeans_kernel_bench.py --rows 100000000 --configs v10:1 --modes 0 --iters 3"
for build in base $V; do
  if [ "$build" = base ]; then lib=$PWD/alink_amd/ops/libalink_hip.so; else lib=$PWD/variants/libalink_hip_$build.so; fi
  ALINK_HIP_LIB=$lib tools/gpu.sh pmc ${build}_mix "$P1" 90 $B || exit 1
  ALINK_HIP_LIB=$lib tools/gpu.sh pmc ${build}_busy "$P2" 90 $B || exit 1
done
find gpurun_out -path '*pmc_*' -name '*counter_collection.csv' | sort | while read -r c; do
  python tools/pmc_summary.py "$c" --match kmeans_v10 >> gpurun_out/pmc_r4_summary.txt 2>&1 || true
done
echo PMC_DONE
