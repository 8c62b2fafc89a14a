set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for args in "--k 100" "--k 100 --load-only" "--k 100 --compute-only" "--k 32" "--k 64" "--k 128" "--k 100 --grid 512"; do
  timeout -k 10 120 python tools/kmeans_kernel_bench.py --rows 100000000 --iters 7 $args >> gpurun_out/v7_diag.log 2>&1 || exit 1
done
cat gpurun_out/v7_diag.log
