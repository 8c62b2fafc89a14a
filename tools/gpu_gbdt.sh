set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_tree.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_tree.log 2>&1 && echo TREE_TESTS_OK || { tail -50 gpurun_out/pytest_tree.log; exit 1; }
tail -1 gpurun_out/pytest_tree.log
timeout -k 10 300 python tools/gbdt_bench.py --rows 2000000 --features 1000 --trees 5 --depth 8 --dtype float32 2>&1 | tail -1 | tee gpurun_out/gbdt_mid.json || exit 1
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_gbdt -o gbdt -- python3 $R/tools/gbdt_bench.py --rows 2000000 --features 1000 --trees 5 --depth 8 --dtype float32 > $R/gpurun_out/prof_gbdt.log 2>&1 && echo PROF_OK || { tail -5 $R/gpurun_out/prof_gbdt.log; exit 1; }
cd $R && timeout -k 10 900 python tools/gbdt_bench.py --rows 20000000 --features 1000 --trees 20 --depth 8 --dtype float32 2>&1 | tail -1 | tee gpurun_out/gbdt_big.json
