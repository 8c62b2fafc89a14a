set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_als.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_als.log 2>&1 && echo ALS_TESTS_OK || { tail -40 gpurun_out/pytest_als.log; exit 1; }
export ALINK_ALS_PROFILE=1
timeout -k 10 900 python -u tools/als_bench.py > gpurun_out/als_big.log 2>&1 && tail -1 gpurun_out/als_big.log || { tail -5 gpurun_out/als_big.log; exit 1; }
