# dense linear gradient tests (narrow + wide d) and bandwidth sweep, then GBDT at 1000 features (config-3 shape)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kmeans_kernel_gpu.py -q -x -k linear_grad --timeout 120 --timeout-method thread > gpurun_out/linear_tests.log 2>&1; rc=$?; tail -3 gpurun_out/linear_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python tools/linear_kernel_bench.py 20000000 > gpurun_out/linear_bench.json 2>&1 && cat gpurun_out/linear_bench.json || exit 1
timeout -k 10 300 python tools/gbdt_bench.py --rows 2000000 --features 1000 --trees 5 --depth 8 --dtype float32 2>&1 | tail -1 | tee gpurun_out/gbdt_mid.json || exit 1
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_gbdt -o gbdt -- python3 $R/tools/gbdt_bench.py --rows 2000000 --features 1000 --trees 5 --depth 8 --dtype float32 > $R/gpurun_out/prof_gbdt.log 2>&1 && echo PROF_OK || { tail -5 $R/gpurun_out/prof_gbdt.log; exit 1; }
cd $R && timeout -k 10 700 python tools/gbdt_bench.py --rows 20000000 --features 1000 --trees 20 --depth 8 --dtype float32 2>&1 | tail -1 | tee gpurun_out/gbdt_big.json
