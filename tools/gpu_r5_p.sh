#!/bin/bash
# round-5 GPU call: FTRL pipeline host profile after the block scan
set -o pipefail
tools/gpu.sh run ftrl_cprof 300 python -m cProfile -o gpurun_out/ftrl.prof tools/ftrl_pipeline_bench.py --rows 16000000 || exit 1
