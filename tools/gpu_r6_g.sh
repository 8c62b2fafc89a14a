#!/bin/bash
# round-6: does the bench's own instrumentation (per-launch HIP events, the amdsmi sampler) cost time at the
# 8-GPU per-rank shape (1.25e7 rows)?  Alternating runs on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for kt in 1 0; do
    for tel in 1 0; do
      echo "== round $r kernel_timing $kt telemetry $tel"
      timeout -k 10 150 python -u bench.py --rows 12500000 --steps 100 --warmup 5 --converge-iters 0 \
        --kernel-timing $kt --telemetry $tel | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d.get('assign_ms_per_step_max'))" || exit 1
    done
  done
done
