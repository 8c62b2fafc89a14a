#!/bin/bash
# round-5 GPU call: f64 MFMA lane maps / throughput probe; ALS baseline kernel table before the MFMA Gram
set -o pipefail
R=$PWD
tools/gpu.sh run mfma_f64 60 tools/micro/mfma_f64_probe || exit 1
tools/gpu.sh prof als 400 python $R/tools/als_bench.py --iters 2 || exit 1
python tools/rocpd_stats.py gpurun_out/prof_als/als_results.db --top 20 > gpurun_out/prof_als_stats.txt 2>&1 || true
find gpurun_out -type f -size +1M ! -name '*.gz' -exec gzip -9 {} \;
