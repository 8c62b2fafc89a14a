#!/bin/bash
# round-5 GPU call: ALS user sweep (Woodbury 9..16 ratings) on the f64 matrix cores; KMeans convergence-run split;
# RF levels after RowOrder; FTRL scoring path
set -o pipefail
R=$PWD
LIMIT=500 tools/gpu.sh tests tests/test_als.py tests/test_ftrl_gpu.py tests/test_linear_gpu.py tests/test_oneshot_gpu.py || exit 1
ALINK_ALS_WOODBURY_MFMA=1 tools/gpu.sh prof als 400 python $R/tools/als_bench.py --iters 2 || exit 1
python tools/rocpd_stats.py gpurun_out/prof_als/als_results.db --top 20 > gpurun_out/prof_als_stats.txt 2>&1 || true
ALINK_ALS_WOODBURY_MFMA=1 ALINK_ALS_WOODBURY_BUCKETS=16,32 tools/gpu.sh run als_b16 300 python tools/als_bench.py --iters 2 || exit 1
ALINK_ALS_WOODBURY_MFMA=0 tools/gpu.sh run als_lds 300 python tools/als_bench.py --iters 2 || exit 1
tools/gpu.sh run initprof 300 python tools/kmeans_init_profile.py --reps 2 || exit 1
tools/gpu.sh run rflevels 600 python tools/rf_level_bench.py --rows 1000000 --features 100 || exit 1
tools/gpu.sh run ftrl32 300 python tools/ftrl_pipeline_bench.py --rows 32000000 || exit 1
tools/gpu.sh prof ftrl 300 python $R/tools/ftrl_pipeline_bench.py --rows 8000000 || exit 1
python tools/rocpd_stats.py gpurun_out/prof_ftrl/ftrl_results.db --top 25 > gpurun_out/prof_ftrl_stats.txt 2>&1 || true
find gpurun_out -type f -size +1M ! -name '*.gz' -exec gzip -9 {} \;
