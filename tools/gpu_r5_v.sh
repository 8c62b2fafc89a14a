#!/bin/bash
# round-5 GPU call: 8-process one-GPU rehearsal of the headline KMeans after the one-shot poll back-off,
# compared with the 1-rank model of the same scenario
set -o pipefail
R=$PWD
tools/gpu.sh run reh1 200 env ALINK_ONESHOT_TIMEOUT_S=60 python tools/mp_rehearsal.py --world 1 --scenario kmeans_headline --out gpurun_out/reh1 --timeout 150 || exit 1
tools/gpu.sh run reh8 330 env ALINK_ONESHOT_TIMEOUT_S=60 python tools/mp_rehearsal.py --world 8 --scenario kmeans_headline --out gpurun_out/reh8 --timeout 300 --compare gpurun_out/reh1/kmeans_headline_1_0.json
find gpurun_out -type f -size +4M ! -name '*.gz' -exec gzip -9 {} \;
