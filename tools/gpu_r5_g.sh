#!/bin/bash
# round-5 GPU call: full GPU suite, discretizer / Spearman at 1e8, RF per-level timing
set -o pipefail
LIMIT=900 tools/gpu.sh tests tests/ || exit 1
tools/gpu.sh run discretizer 300 python tools/discretizer_bench.py --rows 100000000 --buckets 100 || exit 1
tools/gpu.sh run rflevels 600 python tools/rf_level_bench.py --rows 1000000 --features 100 || exit 1
