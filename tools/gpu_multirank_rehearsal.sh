# 2 and 4 ranks on ONE MI355X with the gloo backend (RCCL cannot put two ranks on one GPU): exercises the
# self-launcher, speculative supersteps, barrier-bracketed timing and the collectives of bench.py at N > 1
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 2 4; do
ALINK_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus $n --steps 5 --warmup 2 --rows 20000000 --converge-iters 5 > gpurun_out/bench_rehearsal_$n.log 2>&1 && tail -1 gpurun_out/bench_rehearsal_$n.log || { tail -30 gpurun_out/bench_rehearsal_$n.log; exit 1; }
done
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --rows 20000000 --converge-iters 5 > gpurun_out/bench_rehearsal_1.log 2>&1 && tail -1 gpurun_out/bench_rehearsal_1.log
