#!/bin/bash
# round-5 GPU call: KMeans v10 work-stealing tail (DYN) — tests, per-workgroup timeline, A/B, benches
set -o pipefail
LIMIT=300 tools/gpu.sh tests tests/test_kmeans_kernel_gpu.py  || exit 1
ALINK_HIP_LIB=variants/libalink_hip_timing.so tools/gpu.sh run wgtiming 200 python tools/kmeans_wg_timing.py --rows 12500000,100000000 || exit 1
tools/gpu.sh run kbench 400 python tools/kmeans_kernel_bench.py --rows 100000000 --sub-rows 12500000 --configs v10:1ap0,v10:1ap0.05,v10:1ap0.1,v10:1ap0.2,v10:1ap0,v10:1ap0.1 --iters 20 || exit 1
TAG=bench_r125 LIMIT=200 tools/gpu.sh bench --rows 12500000 --steps 50 --warmup 5 --converge-iters 0 || exit 1
ALINK_KMEANS_V10_POOL=0 TAG=bench_r125_static LIMIT=200 tools/gpu.sh bench --rows 12500000 --steps 50 --warmup 5 --converge-iters 0 || exit 1
LIMIT=300 tools/gpu.sh bench || exit 1
