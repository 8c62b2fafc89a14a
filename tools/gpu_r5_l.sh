#!/bin/bash
# round-5 GPU call: FTRL pipeline kernel trace after the device-resident scoring -> evaluation path
set -o pipefail
R=$PWD
tools/gpu.sh prof ftrl 300 python $R/tools/ftrl_pipeline_bench.py --rows 8000000 || exit 1
python tools/rocpd_stats.py gpurun_out/prof_ftrl/ftrl_results.db --top 25 > gpurun_out/prof_ftrl_stats.txt 2>&1 || true
find gpurun_out -type f -size +1M ! -name '*.gz' -exec gzip -9 {} \;
