#!/bin/bash
# round-4 GPU call B: FTRL stream pipeline (SHARDED, DATA_PARALLEL async), fp32 KMeans path, GBDT quantize
# profile, then the 8-process one-GPU rehearsal of the headline KMeans (last: the longest and riskiest step)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tools/gpu.sh run ftrl_pipe_sharded 240 python tools/ftrl_pipeline_bench.py --mode SHARDED || exit 1
tools/gpu.sh run ftrl_pipe_dp 240 python tools/ftrl_pipeline_bench.py --mode DATA_PARALLEL --async-reduce || exit 1
tools/gpu.sh run kmeans_fp32 200 python tools/kmeans_fp32_bench.py || exit 1
tools/gpu.sh prof gbdt_q 300 python tools/gbdt_bench.py --rows 20000000 --features 1000 --trees 2 --depth 8 --dtype float32 --ranks 1 || exit 1
tools/gpu.sh run reh8 330 env ALINK_ONESHOT_TIMEOUT_S=60 python tools/mp_rehearsal.py --world 8 --scenario kmeans_headline --out gpurun_out/reh8 --timeout 300
