#!/bin/bash
# round-5 GPU call: host profiles of the FTRL StreamOp pipeline and of a deep random forest
set -o pipefail
tools/gpu.sh run ftrl32 300 python tools/ftrl_pipeline_bench.py --rows 32000000 || exit 1
tools/gpu.sh run ftrl_cprof 300 python -m cProfile -o gpurun_out/ftrl.prof tools/ftrl_pipeline_bench.py --rows 16000000 || exit 1
python tools/prof_print.py gpurun_out/ftrl.prof 45 > gpurun_out/ftrl_prof.txt 2>&1 || true
tools/gpu.sh run rf_cprof 300 python -m cProfile -o gpurun_out/rf.prof tools/rf_level_bench.py --rows 1000000 --features 100 || exit 1
python tools/prof_print.py gpurun_out/rf.prof 40 > gpurun_out/rf_prof.txt 2>&1 || true
