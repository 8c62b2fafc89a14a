#!/bin/bash
# round-5 GPU call: bench order A/B (convergence runs after / before the timed run)
set -o pipefail
for i in 1 2; do
  TAG=ord_a_$i tools/gpu.sh bench --steps 20 --warmup 5 || exit 1
  TAG=ord_b_$i tools/gpu.sh bench --steps 20 --warmup 5 --convergence-first 1 || exit 1
done
