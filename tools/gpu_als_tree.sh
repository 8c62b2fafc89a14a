set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_als.py tests/test_tree.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_als_tree.log 2>&1 && echo TESTS_OK || { tail -50 gpurun_out/pytest_als_tree.log; exit 1; }
tail -1 gpurun_out/pytest_als_tree.log
timeout -k 10 300 python tools/gbdt_bench.py --rows 2000000 --features 1000 --trees 5 --depth 8 --dtype float32 2>&1 | tail -1 | tee gpurun_out/gbdt_mid2.json || exit 1
timeout -k 10 300 python tools/als_bench.py --users 1000000 --items 100000 --ratings 10000000 2>&1 | tail -1 | tee gpurun_out/als_small.json || exit 1
timeout -k 10 600 python tools/als_bench.py 2>&1 | tail -1 | tee gpurun_out/als_big.json
