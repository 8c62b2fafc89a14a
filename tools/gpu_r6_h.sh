#!/bin/bash
# round-6: bench.py at the 8-GPU per-rank shape, the round-5 tree (variants/r5tree, built in place) vs HEAD,
# alternating on one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for tree in variants/r5tree .; do
    echo "== round $r tree $tree"
    (cd $tree && timeout -k 10 150 python -u bench.py --rows 12500000 --steps 100 --warmup 5 --converge-iters 0) \
      | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])" || exit 1
  done
done
for r in 1 2; do
  for tree in variants/r5tree .; do
    echo "== 1e8 round $r tree $tree"
    (cd $tree && timeout -k 10 150 python -u bench.py --steps 20 --warmup 3 --converge-iters 0) \
      | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])" || exit 1
  done
done
