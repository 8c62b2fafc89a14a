# full GPU check: gpu tests, smoke, 1-GPU bench (JSON -> gpurun_out/bench.json), rocprofv3 kernel stats of the bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && echo PYTEST_OK || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK || { tail -30 gpurun_out/smoke.log; exit 1; }
timeout -k 10 500 python bench.py --steps 20 --warmup 3 > gpurun_out/bench.log 2>&1 && echo BENCH_OK || { tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log > gpurun_out/bench.json; cat gpurun_out/bench.json
if [ "${PROF:-0}" = 1 ]; then
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --converge-iters 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.log 2>&1 && echo PROF_OK
fi
