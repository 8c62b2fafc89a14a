set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kmeans_general_gpu.py -q -x --timeout 200 --timeout-method thread > gpurun_out/kmgen_tests.log 2>&1; rc=$?; tail -15 gpurun_out/kmgen_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 python tools/kmeans_general_bench.py > gpurun_out/kmgen_bench.log 2>&1; rc=$?; cat gpurun_out/kmgen_bench.log | grep -v amdgpu.ids; exit $rc
