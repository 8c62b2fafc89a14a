# tree kernels on the GPU: gpu tests for the tree family, GBDT throughput (both histogram kernels), rocprof
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_tree.py -x -q -m gpu > gpurun_out/pytest_tree_gpu.log 2>&1 && echo PYTEST_OK || { tail -40 gpurun_out/pytest_tree_gpu.log; exit 1; }
for v in 0 1; do
ALINK_TREE_HIST_VARIANT=$v timeout -k 10 300 python tools/gbdt_bench.py --rows 20000000 --features 28 --trees 20 --depth 6 > gpurun_out/gbdt_bench_v$v.log 2>&1 && tail -1 gpurun_out/gbdt_bench_v$v.log || { tail -40 gpurun_out/gbdt_bench_v$v.log; exit 1; }
done
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_tree -o run -- python3 $R/tools/gbdt_bench.py --rows 10000000 --features 28 --trees 5 --depth 6 > $R/gpurun_out/gbdt_prof.log 2>&1 || { tail -30 $R/gpurun_out/gbdt_prof.log; exit 1; }
find /tmp/prof_tree -name "*kernel_stats.csv" -exec cp {} $R/gpurun_out/gbdt_kernel_stats.csv \;
cut -c1-60,400- $R/gpurun_out/gbdt_kernel_stats.csv | head -12
