#!/bin/bash
# round-5 GPU call: ALS light rows on the f64 matrix cores (als_mfma_solve); FTRL whole-segment block scan
set -o pipefail
R=$PWD
LIMIT=500 tools/gpu.sh tests tests/test_als.py tests/test_ftrl_gpu.py || exit 1
tools/gpu.sh prof als 400 python $R/tools/als_bench.py --iters 2 || exit 1
python tools/rocpd_stats.py gpurun_out/prof_als/als_results.db --top 20 > gpurun_out/prof_als_stats.txt 2>&1 || true
tools/gpu.sh run ftrl32 300 python tools/ftrl_pipeline_bench.py --rows 32000000 || exit 1
find gpurun_out -type f -size +1M ! -name '*.gz' -exec gzip -9 {} \;
