# all tests on the GPU box: CPU-marked tests then run with the default device = cuda:0 (device-resident paths)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -q -x -m gpu > gpurun_out/pytest_gpu.log 2>&1 && echo GPU_TESTS_OK || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 900 python -m pytest tests -q -m "not gpu" -p no:cacheprovider > gpurun_out/pytest_cpu_on_gpu.log 2>&1; echo "cpu-suite-on-gpu rc=$?"; tail -30 gpurun_out/pytest_cpu_on_gpu.log
