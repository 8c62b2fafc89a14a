set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_e2e_gpu.py tests/test_linear_gpu.py tests/test_examples.py -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_e2e.log 2>&1; rc=$?
tail -40 gpurun_out/pytest_e2e.log | grep -v "^$" | tail -30
exit $rc
