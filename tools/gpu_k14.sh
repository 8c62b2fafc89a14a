set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kmeans_kernel_gpu.py tests/test_linear.py tests/test_e2e_gpu.py -q -x -k "search or linear or logistic or Linear or Logistic or svm or Svm" --timeout 200 --timeout-method thread > gpurun_out/k14_tests.log 2>&1; rc=$?; tail -5 gpurun_out/k14_tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python tools/lr_train_bench.py > gpurun_out/lr_bench.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/lr_bench.log; exit $rc
