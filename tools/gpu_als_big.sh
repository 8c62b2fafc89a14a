set -o pipefail
export TMPDIR=/tmp
export ALINK_ALS_PROFILE=1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/als_bench.py --users 1000000 --items 100000 --ratings 10000000 > gpurun_out/als_small.log 2>&1 && tail -1 gpurun_out/als_small.log || { tail -5 gpurun_out/als_small.log; exit 1; }
timeout -k 10 900 python -u tools/als_bench.py > gpurun_out/als_big.log 2>&1 && tail -1 gpurun_out/als_big.log || { tail -5 gpurun_out/als_big.log; exit 1; }
