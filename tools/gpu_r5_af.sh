#!/bin/bash
# round-5 GPU call: PMC of the k-means|| weights pass (nearest kernel counts mode, 201 candidates, 1e8 x 128)
set -o pipefail
R=$PWD
export NEAREST_ONLY_M=201
tools/gpu.sh pmc near1 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" 90 python $R/tools/kmeans_nearest_bench.py --reps 3 || exit 1
tools/gpu.sh pmc near2 "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE" 90 python $R/tools/kmeans_nearest_bench.py --reps 3 || exit 1
python tools/pmc_summary.py $(find gpurun_out/pmc_near1 gpurun_out/pmc_near2 -name "*counter_collection.csv") --match kmeans_nearest > gpurun_out/pmc_near_summary.txt 2>&1 || true
