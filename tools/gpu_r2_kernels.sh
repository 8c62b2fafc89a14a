# round-2 kernel batch: colstats (K23), FM (K18), W2V (K20), top-K (K28) GPU tests
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_colstats_gpu.py tests/test_fm_gpu.py tests/test_w2v_gpu.py tests/test_lda_gpu.py tests/test_topk_gpu.py tests/test_lda.py tests/test_fm.py tests/test_nlp.py -x -v -s -m gpu --timeout 120 --timeout-method thread > gpurun_out/r2k_tests.log 2>&1 && echo TESTS_OK || { tail -60 gpurun_out/r2k_tests.log; exit 1; }
grep -E "colstats 4e6|passed|failed" gpurun_out/r2k_tests.log
