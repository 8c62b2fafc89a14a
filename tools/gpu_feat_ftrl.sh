set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_feature_gpu.py tests/test_ftrl_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_feat_ftrl.log 2>&1 && echo TESTS_OK || { tail -60 gpurun_out/pytest_feat_ftrl.log; exit 1; }
tail -2 gpurun_out/pytest_feat_ftrl.log
timeout -k 10 300 python tools/ftrl_bench.py > gpurun_out/ftrl_bench.json 2> gpurun_out/ftrl_bench.err && cat gpurun_out/ftrl_bench.json || { tail -20 gpurun_out/ftrl_bench.err; exit 1; }
