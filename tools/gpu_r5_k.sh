#!/bin/bash
# round-5 GPU call: device-resident scoring -> evaluation; FTRL pipeline throughput
set -o pipefail
LIMIT=400 tools/gpu.sh tests tests/test_ftrl_gpu.py tests/test_linear_gpu.py tests/test_evaluation.py tests/test_e2e_gpu.py || exit 1
tools/gpu.sh run ftrl32 300 python tools/ftrl_pipeline_bench.py --rows 32000000 || exit 1
tools/gpu.sh run ftrl_cprof 300 python -m cProfile -o gpurun_out/ftrl.prof tools/ftrl_pipeline_bench.py --rows 16000000 || exit 1
