set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/variants.log
for st in "--compute-only" ""; do timeout -k 10 200 python tools/kmeans_kernel_bench.py --rows 100000000 --k 100 --iters 7 --variant 6 $st >> gpurun_out/variants.log 2>&1 || exit 1; done
grep rows gpurun_out/variants.log | cut -c1-220
