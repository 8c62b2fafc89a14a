#!/bin/bash
# round-4 GPU call D: FTRL pipeline with frequent snapshots (model updates reach the predictor), GBDT quantize
# profile, then the 8-process one-GPU rehearsal of the headline KMeans (last: the longest step)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
tools/gpu.sh run ftrl_pipe_sharded_32m 240 python tools/ftrl_pipeline_bench.py --mode SHARDED --rows 32000000 || exit 1
tools/gpu.sh run ftrl_pipe_dp_32m 240 python tools/ftrl_pipeline_bench.py --mode DATA_PARALLEL --async-reduce --rows 32000000 || exit 1
tools/gpu.sh prof ftrl_pipe 240 python $R/tools/ftrl_pipeline_bench.py --mode SHARDED --rows 8000000 || exit 1
tools/gpu.sh prof gbdt_q 300 python $R/tools/gbdt_bench.py --rows 20000000 --features 1000 --trees 2 --depth 8 --dtype float32 --ranks 1 || exit 1
tools/gpu.sh run reh8 330 env ALINK_ONESHOT_TIMEOUT_S=60 python tools/mp_rehearsal.py --world 8 --scenario kmeans_headline --out gpurun_out/reh8 --timeout 300
rc=$?
find gpurun_out -type f -size +1M ! -name '*.gz' -exec gzip -9 {} \;
du -sh gpurun_out
exit $rc
